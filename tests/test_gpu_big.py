"""Worlds above 1024 agents per env: the reference steps any sum(n_agents)
(gym_macm/envs/mvmnt.py:61) in one uncapped b2World. Here an env of 1024 < N <= 4096 agents is one
workgroup of 1024 threads with up to 4 bodies per thread (csrc/flock_big.hip: the spill step, its
HBM working set, the island DFS, and Gauss-Seidel levels stepped by one wave). Bar: bit-exact against the
oracle (oracle/, the C restatement of mvmnt.py over b2lite) in state, contact lists, rewards,
neighbour ids, done, reward sums, and the observation within the f32 tolerance of tests/parity.py,
sparse and dense, through the tensor API (step, rollout, trajectory, per-env resets) and the dict API.
Speed is not the point here (no BASELINE config exceeds 1024 agents)."""
import random

import numpy as np
import pytest
import torch

from parity import assert_state_equal, f32_obs_mismatch
from test_gpu_parity import check_rollout, make_pair, rand_actions

pytestmark = pytest.mark.gpu

from gym_macm.settings import flockSettings, to_config  # noqa: E402


@pytest.mark.parametrize("E,N,spread,steps,kw", [
    (2, 1500, 60.0, 12, {}),                                           # sparse, 2 bodies per thread
    (2, 1100, 30.0, 10, {"reward_mode": "linear", "coord": "cartesian"}),  # a partial second chunk
    (1, 2048, 20.0, 6, {}),                                            # dense: one island of thousands
    (1, 4096, 90.0, 5, {}),                                            # 4 bodies per thread
])
def test_big_world_matches_oracle(E, N, spread, steps, kw):
    vec, orc = make_pair(E, [N], seed=N + E, start_spread=spread, **kw)
    assert vec.world.C >= 1
    check_rollout(vec, orc, steps, np.random.default_rng(N), state_every=max(1, steps // 2))
    assert vec.status() == 0


def test_big_world_two_flocks_f64_obs():
    E, N = 2, 1300
    targets = [0] * 650 + [1] * 650
    vec, orc = make_pair(E, [650, 650], seed=77, targets=targets, obs_dtype=torch.float64, start_spread=50.0)
    check_rollout(vec, orc, 8, np.random.default_rng(3), state_every=4, obs_f64=True)


def test_big_world_rollout_trajectory_and_reset_envs():
    """One trajectory launch of K steps equals the oracle's K steps row by row; then per-env resets
    continue each env's own MT19937 stream (macm_world_reset_envs with the big init kernel)."""
    E, N, K = 2, 1200, 6
    vec, orc = make_pair(E, [N], seed=5, start_spread=40.0)
    rng = np.random.default_rng(9)
    acts = np.stack([rand_actions(rng, E, N) for _ in range(K)])
    traj = vec.rollout(torch.from_numpy(acts).cuda(), trajectory=True)
    for k in range(K):
        r = orc.step(acts[k])
        np.testing.assert_array_equal(traj["reward"][k].cpu().numpy(), r["reward"].astype(np.float32))
        np.testing.assert_array_equal(traj["nbr_id"][k].cpu().numpy(), r["nbr_id"])
        f32_obs_mismatch(traj["obs"][k].cpu().numpy(), r["obs"])
    assert_state_equal(vec.get_state(), orc.get_state(vec.world.C), "after the trajectory")
    mask = np.array([1, 0], np.uint8)
    vec.reset_envs(torch.from_numpy(mask).cuda())
    orc.reset_envs(mask)
    assert_state_equal(vec.get_state(), orc.get_state(vec.world.C), "after reset_envs")
    check_rollout(vec, orc, 3, rng)


def test_big_world_dict_api():
    """gym_macm.envs.Flock(n_agents=[1500]) through the dict API against the oracle env built after the
    same random.seed (the reference's draw order, mvmnt.py:47-64)."""
    from gym_macm.envs import Flock
    from oracle import OracleFlock
    seed, N = 99, 1500
    random.seed(seed)
    env = Flock(n_agents=[N], device="cuda:0", start_spread=45)
    orc = OracleFlock(to_config(flockSettings(start_spread=45), N, 1, obs_f64=True), None, 1, seed)
    rng = np.random.default_rng(2)
    for t in range(4):
        a = rand_actions(rng, 1, N)
        obs, rewards = env.step({i: a[0, i].astype(np.int64) for i in range(N)})
        r = orc.step(a)
        exp = [int(v) if v != -1 else -1 for v in r["reward"][0]]
        assert [rewards[i] for i in range(N)] == exp, f"rewards step {t}"
        np.testing.assert_array_equal([obs[i]["nodes"][0]["id"] for i in range(N)], r["nbr_id"][0])
    assert_state_equal(env.world.get_state(), orc.get_state(env.world.C), "dict api")


# ---- TDM above 1024 agents (combat.py:82-83 takes any team sizes) ----------------------------------

@pytest.mark.parametrize("teams,side,steps", [
    ([700, 700], 140.0, 6),          # 2 agents per thread, sparse
    ([600, 500], 40.0, 4),           # crowded: deaths-free but many touching contacts
    ([1500, 1500], 300.0, 3),        # 3000 agents: 4 per thread
])
def test_big_tdm_matches_oracle(teams, side, steps):
    from test_gpu_tdm import check_rollout as tdm_check, make_pair as tdm_pair, random_actions
    E, N = 1, sum(teams)
    w, orc = tdm_pair(E, teams, seed=N, world_width=side, world_height=side)
    rng = np.random.default_rng(N)
    tdm_check(w, orc, steps, lambda o, m: random_actions(rng, E, N, p_attack=0.5), state_every=max(1, steps // 2))


def test_big_tdm_dict_api():
    """The drop-in TDM dict API (the reference's 30 x 30 world, combat.py:76-77) with 550 + 500 agents:
    a packed world through the workgroup step with 2 agents per thread; every alive agent sees every
    other alive agent."""
    from gym_macm.envs import TDM
    env = TDM(n_agents=[550, 500])
    assert len(env.agents) == 1050
    rng = np.random.default_rng(1)
    for _ in range(2):
        acts = {aid: np.array([rng.integers(3), rng.integers(3), rng.integers(3), rng.integers(2)])
                for aid in env.obs}
        obs = env.step(acts)
        for aid, o in list(obs.items())[:50]:
            assert len(o["agents"]) == len(obs) - 1
