"""TDM on the HIP path vs the CPU oracle and the reference goldens, through the C-ABI.

Bar: bit-exact for positions, velocities, angles, fat AABBs, sleep clocks, the
ordered contact list with warm-start impulses, health, cooldowns, alive, the
listener, done and winner; observations (float32) equal the oracle's f64 values
rounded to f32 with at most 1 ulp where double atan2 of ocml and glibc round
differently; float64 observations within a few ulp (same reason)."""
import numpy as np
import pytest
import torch

import goldens
from oracle import OracleTDM
from parity import combat_bot, f32_obs_mismatch
from test_oracle_tdm_golden import tdm_obs_close

pytestmark = pytest.mark.gpu

from gym_macm.tdm_world import TdmWorld, tdm_config  # noqa: E402

STATE_KEYS = ("pos", "vel", "angle", "fat", "sleep", "health", "cd_atk", "cd_mov", "alive", "listener",
              "step_count", "time_passed", "done", "winner")


def assert_tdm_state_equal(gs, os_, ctx=""):
    for k in STATE_KEYS:
        np.testing.assert_array_equal(gs[k], os_[k], err_msg=f"{ctx} state[{k}]")
    np.testing.assert_array_equal(gs["contact_count"], os_["contact_count"], err_msg=f"{ctx} contact_count")
    for e in range(gs["contact_count"].shape[0]):
        n = int(gs["contact_count"][e])
        np.testing.assert_array_equal(gs["contact_ab"][e, :n], os_["contact_ab"][e, :n],
                                      err_msg=f"{ctx} env {e} contact order")
        np.testing.assert_array_equal(gs["contact_imp"][e, :n], os_["contact_imp"][e, :n],
                                      err_msg=f"{ctx} env {e} impulses")


def make_pair(E, n_agents, seed, env_offset=0, obs_f64=False, **kw):
    cfg = tdm_config(n_agents, obs_f64=obs_f64, **kw)
    w = TdmWorld(cfg, E, device="cuda:0")
    w.reset(seed, env_offset)
    ocfg = tdm_config(n_agents, obs_f64=True, **kw)
    orc = OracleTDM(ocfg, E, seed, env_offset)
    return w, orc


def random_actions(rng, E, N, p_attack=0.5):
    a = rng.integers(0, 3, size=(E, N, 4)).astype(np.uint8)
    a[..., 3] = rng.random((E, N)) < p_attack
    return a


def check_obs(w, o_obs, o_mask, ctx):
    if w.cfg.obs_f64:
        for e in range(w.E):
            assert tdm_obs_close(w.obs[e].cpu().numpy(), o_obs[e], o_mask[e]), f"obs {ctx} env {e}"
    else:
        f32_obs_mismatch(w.obs.cpu().numpy(), o_obs)


def check_rollout(w, orc, steps, policy, state_every=1):
    E, N = w.E, w.N
    assert_tdm_state_equal(w.get_state(), orc.get_state(), "reset")
    w.observe()
    o_obs, o_mask = orc.observe()
    np.testing.assert_array_equal(w.mask.cpu().numpy(), o_mask)
    check_obs(w, o_obs, o_mask, "reset")
    for t in range(steps):
        a = policy(o_obs, o_mask)
        w.step(torch.from_numpy(a).cuda())
        r = orc.step(a)
        o_obs, o_mask = r["obs"], r["mask"]
        np.testing.assert_array_equal(w.health.cpu().numpy(), r["health"], err_msg=f"health step {t}")
        np.testing.assert_array_equal(w.alive.cpu().numpy(), r["alive"], err_msg=f"alive step {t}")
        np.testing.assert_array_equal(w.done.cpu().numpy(), r["done"], err_msg=f"done step {t}")
        np.testing.assert_array_equal(w.winner.cpu().numpy(), r["winner"], err_msg=f"winner step {t}")
        np.testing.assert_array_equal(w.mask.cpu().numpy(), r["mask"], err_msg=f"mask step {t}")
        check_obs(w, r["obs"], r["mask"], f"step {t}")
        if (t + 1) % state_every == 0 or t == steps - 1:
            assert_tdm_state_equal(w.get_state(), orc.get_state(), f"step {t}")
    assert w.status() == 0
    return r


def test_tdm_reset_matches_reference_rng():
    w, orc = make_pair(8, [16, 16], seed=99)
    assert_tdm_state_equal(w.get_state(), orc.get_state(), "reset")


@pytest.mark.parametrize("name", goldens.tdm_names())
def test_tdm_goldens_through_hip(name):
    """Replays the reference's own TDM rollouts (combat.py, bots.combat / random
    actions) on the HIP path: every recorded quantity matches."""
    g = goldens.load(name)
    cfg = goldens.tdm_config(g, obs_f64=True)
    w = TdmWorld(cfg, 1, device="cuda:0")
    w.place(g["init_pos"][None], g["init_angle"][None])
    np.testing.assert_array_equal(w.mask[0].cpu().numpy(), g["init_mask"])
    assert tdm_obs_close(w.obs[0].cpu().numpy(), g["init_obs"], g["init_mask"])
    for t in range(g["meta"]["steps"]):
        w.step(torch.from_numpy(g["actions"][t][None]).cuda())
        s = w.get_state()
        np.testing.assert_array_equal(s["pos"][0], g["pos"][t], err_msg=f"pos step {t}")
        np.testing.assert_array_equal(s["angle"][0], g["angle"][t], err_msg=f"angle step {t}")
        np.testing.assert_array_equal(s["health"][0], g["health"][t], err_msg=f"health step {t}")
        np.testing.assert_array_equal(s["alive"][0], g["alive"][t], err_msg=f"alive step {t}")
        np.testing.assert_array_equal(s["cd_atk"][0], g["cd_atk"][t], err_msg=f"cd_atk step {t}")
        np.testing.assert_array_equal(s["cd_mov"][0], g["cd_mov"][t], err_msg=f"cd_mov step {t}")
        np.testing.assert_array_equal(s["listener"][0], g["listener"][t], err_msg=f"listener step {t}")
        assert int(w.done[0]) == int(g["done"][t]) and int(w.winner[0]) == int(g["winner"][t]), t
        np.testing.assert_array_equal(w.mask[0].cpu().numpy(), g["mask"][t], err_msg=f"mask step {t}")
        assert tdm_obs_close(w.obs[0].cpu().numpy(), g["obs"][t], g["mask"][t]), f"obs step {t}"


def test_tdm_bots_rollout_bit_exact():
    """C4 shape (2 x 16) driven by the reference's combat bot until teams die out."""
    w, orc = make_pair(24, [16, 16], seed=41)
    r = check_rollout(w, orc, 500, combat_bot, state_every=10)
    assert (r["alive"] == 0).any() and (r["winner"] >= 0).any()


def test_tdm_random_rollout_dense_world():
    # a 12 x 12 spawn area: many contacts, islands and hits
    w, orc = make_pair(16, [16, 16], seed=5, world_width=12.0, world_height=12.0)
    rng = np.random.default_rng(3)
    check_rollout(w, orc, 250, lambda o, m: random_actions(rng, 16, 32), state_every=5)


def test_tdm_four_teams_64_agents_f64_obs():
    w, orc = make_pair(6, [16, 16, 16, 16], seed=8, obs_f64=True)
    check_rollout(w, orc, 200, combat_bot, state_every=20)


def test_tdm_fresh_raycast_and_decaying_penalty():
    w, orc = make_pair(16, [8, 8], seed=13, fresh_raycast=True, decay_mov_penalty=True)
    check_rollout(w, orc, 300, combat_bot, state_every=15)


def test_tdm_state_injection_continues_identically():
    """Oracle state after 60 steps injected into the HIP world; both continue."""
    E, N = 8, 20
    w, orc = make_pair(E, [10, 10], seed=17, world_width=14.0, world_height=14.0)
    obs, mask = orc.observe()
    for _ in range(60):
        r = orc.step(combat_bot(obs, mask))
        obs, mask = r["obs"], r["mask"]
    w.set_state(orc.get_state())
    assert_tdm_state_equal(w.get_state(), orc.get_state(), "injected")
    check_rollout(w, orc, 120, combat_bot, state_every=10)


def test_tdm_counters_and_latching_done():
    E = 32
    w, orc = make_pair(E, [4, 4], seed=2, world_width=8.0, world_height=8.0)
    obs, mask = orc.observe()
    attacks = deaths = 0
    prev_done = np.zeros(E, np.uint8)
    for t in range(400):
        a = combat_bot(obs, mask)
        alive_before = orc.get_state()["alive"].copy()
        cd = orc.get_state()["cd_atk"]
        attacks += int(((a[..., 3] == 1) & (cd <= 0) & (alive_before == 1)).sum())
        w.step(torch.from_numpy(a).cuda())
        r = orc.step(a)
        obs, mask = r["obs"], r["mask"]
        deaths += int((alive_before.astype(int) - r["alive"]).sum())
        d = w.done.cpu().numpy()
        assert (d >= prev_done).all(), "done latches"
        prev_done = d
    c = w.counters()
    assert c[1] == attacks and c[2] == deaths and deaths > 0
    assert (w.winner.cpu().numpy() >= 0).sum() > 0


def _slots(obs, env):
    """Reference-format obs dict -> fixed slots (as tests/golden/make_golden.tdm_slots)."""
    N = len(env.agents)
    o = np.zeros((N, N - 1, 4))
    m = np.zeros((N, N - 1), np.uint8)
    for i, ag in enumerate(env.agents):
        if ag.id not in obs:
            continue
        others = [j for j in range(N) if j != i and env.agents[j].alive]
        for j, d in zip(others, obs[ag.id]["agents"]):
            k = j if j < i else j - 1
            o[i, k, :3] = d["position"]
            o[i, k, 3] = d["type"]
            m[i, k] = 1
    return o, m


@pytest.mark.parametrize("name", goldens.tdm_names())
def test_dropin_tdm_matches_reference_goldens(name):
    """The drop-in dict API (gym_macm.envs.TDM over the HIP world) reproduces the
    reference env's own rollouts: random.seed -> spawn, actor hook or action dicts,
    obs dicts, health, deaths, done and winner."""
    import random
    from gym_macm.envs import TDM
    from parity import combat_bot_dict
    g = goldens.load(name)
    m = g["meta"]
    random.seed(m["seed"])
    actors = None
    if m["policy"] == "combat":
        actors = [[combat_bot_dict] * n for n in m["n_agents"]]
    env = TDM(render=False, n_agents=m["n_agents"], actors=actors, device="cuda:0")
    o, msk = _slots(env.obs, env)
    np.testing.assert_array_equal(msk, g["init_mask"])
    assert tdm_obs_close(o, g["init_obs"], g["init_mask"])
    for t in range(m["steps"]):
        if actors is None:
            acts = {ag.id: g["actions"][t][k].astype(np.int64) for k, ag in enumerate(env.agents) if ag.alive}
            obs = env.step(acts)
        else:
            obs = env.step()
        o, msk = _slots(obs, env)
        np.testing.assert_array_equal(msk, g["mask"][t], err_msg=f"mask step {t}")
        assert tdm_obs_close(o, g["obs"][t], g["mask"][t]), f"obs step {t}"
        np.testing.assert_array_equal([ag.health for ag in env.agents], g["health"][t], err_msg=f"health {t}")
        assert [ag.alive for ag in env.agents] == list(g["alive"][t].astype(bool)), f"alive step {t}"
        assert env.done == bool(g["done"][t]), f"done step {t}"
        assert (env.winner if env.winner is not None else -1) == int(g["winner"][t]), f"winner step {t}"
        assert env.time_passed == g["time_passed"][t]
        assert sorted(obs) == sorted(ag.id for ag in env.agents if ag.alive)
    assert sum(env.n_alive) == int(g["alive"][-1].sum())


def test_host_outputs_equal_device_outputs():
    """The zero-copy pinned-host outputs (dict API) hold the same values as device outputs."""
    E, teams = 4, [6, 6]
    wd = TdmWorld(tdm_config(teams, world_width=8.0, world_height=8.0), E, device="cuda:0")
    wh = TdmWorld(tdm_config(teams, world_width=8.0, world_height=8.0), E, device="cuda:0", host_outputs=True)
    wd.reset(3)
    wh.reset(3)
    rng = np.random.default_rng(0)
    act_h = torch.empty((E, 12, 4), dtype=torch.uint8, pin_memory=True)
    for t in range(60):
        a = random_actions(rng, E, 12)
        wd.step(torch.from_numpy(a).cuda())
        act_h.numpy()[:] = a
        wh.step(act_h)
        torch.cuda.synchronize()
        for x, y in zip(wd.outputs(), wh.outputs()):
            np.testing.assert_array_equal(x.cpu().numpy(), y.numpy(), err_msg=f"step {t}")
