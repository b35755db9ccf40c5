"""Per-env resets on the device (macm_world_reset_envs / macm_tdm_reset_envs) vs the
oracle's reset_envs (next poses from each env's CPython MT19937 stream, fresh
world). Bar: bit-exact states and equal observations, through repeated resets
that cross MT19937 twists, for the wave and workgroup kernels, TDM, and the
done-driven auto-reset."""
import numpy as np
import pytest
import torch

from oracle import OracleTDM
from parity import assert_state_equal, combat_bot, f32_obs_mismatch, oracle_for
from test_gpu_tdm import assert_tdm_state_equal

pytestmark = pytest.mark.gpu

from gym_macm._abi import MacmError  # noqa: E402
from gym_macm.settings import flockSettings, to_config  # noqa: E402
from gym_macm.tdm_world import TdmWorld, tdm_config  # noqa: E402
from gym_macm.vec import FlockVec  # noqa: E402


def flock_pair(E, N, seed, **kw):
    vec = FlockVec(E, n_agents=[N], seed=seed, device="cuda:0", **kw)
    orc = oracle_for(to_config(flockSettings(**{k: v for k, v in kw.items() if k != "autoreset"}), N, 1,
                               obs_f64=True), None, E, seed)
    return vec, orc


@pytest.mark.parametrize("N", [16, 64, 100])
def test_flock_reset_envs_continue_each_stream(N):
    E = 12
    vec, orc = flock_pair(E, N, seed=77, start_spread=12)
    rng = np.random.default_rng(N)
    for rnd in range(5):  # 5 resets of 3N draws: the 624-word MT state twists on the way
        for _ in range(20):
            a = rng.integers(0, 3, size=(E, N, 3)).astype(np.uint8)
            vec.step(torch.from_numpy(a).cuda())
            orc.step(a)
        mask = (rng.random(E) < 0.5).astype(np.uint8)
        mask[rnd % E] = 1
        vec.reset_envs(torch.from_numpy(mask).cuda())
        orc.reset_envs(mask)
        assert_state_equal(vec.get_state(), orc.get_state(vec.world.C), f"reset round {rnd}")
        o, nbr = orc.observe()
        m = mask.astype(bool)
        np.testing.assert_array_equal(vec.nbr_id.cpu().numpy()[m], nbr[m])
        f32_obs_mismatch(vec.obs.cpu().numpy()[m], o[m])
    vec.reset_envs()  # all
    orc.reset_envs()
    assert_state_equal(vec.get_state(), orc.get_state(vec.world.C), "reset all")


def test_flock_autoreset_on_done():
    """hz=60, time_limit=0.25: every env is done at step 16 and restarts; with
    autoreset the device resets on its own done flags, no host round trip."""
    E, N = 8, 32
    vec, orc = flock_pair(E, N, seed=5, time_limit=0.25, autoreset=True)
    rng = np.random.default_rng(0)
    resets = 0
    for t in range(70):
        a = rng.integers(0, 3, size=(E, N, 3)).astype(np.uint8)
        obs, nbr, rew, done = vec.step(torch.from_numpy(a).cuda())
        r = orc.step(a)
        np.testing.assert_array_equal(done.cpu().numpy(), r["done"], err_msg=f"done step {t}")
        np.testing.assert_array_equal(rew.cpu().numpy(), r["reward"].astype(np.float32), err_msg=f"rew {t}")
        if r["done"].any():
            orc.reset_envs(r["done"])
            resets += 1
        assert_state_equal(vec.get_state(), orc.get_state(vec.world.C), f"step {t}")
    assert resets == 4


def test_reset_envs_needs_device_streams():
    vec, _ = flock_pair(2, 8, seed=1)
    vec.world.place(np.zeros((2, 8, 2), np.float32) + np.arange(8)[None, :, None] * 2,
                    np.zeros((2, 8), np.float32), np.ones((2, 1, 2), np.float32))
    with pytest.raises(MacmError):
        vec.reset_envs()


def test_tdm_reset_envs_and_autoreset_on_done():
    E, teams = 16, [4, 4]
    cfg = dict(world_width=8.0, world_height=8.0)
    w = TdmWorld(tdm_config(teams, **cfg), E, device="cuda:0")
    w.reset(31)
    orc = OracleTDM(tdm_config(teams, obs_f64=True, **cfg), E, 31)
    obs, mask = orc.observe()
    resets = 0
    for t in range(600):
        a = combat_bot(obs, mask)
        w.step(torch.from_numpy(a).cuda())
        r = orc.step(a)
        if r["done"].any():
            w.reset_envs(w.done)
            orc.reset_envs(r["done"])
            resets += int(r["done"].sum())
        obs, mask = orc.observe()
        if t % 20 == 19:
            assert_tdm_state_equal(w.get_state(), orc.get_state(), f"step {t}")
    assert_tdm_state_equal(w.get_state(), orc.get_state(), "end")
    np.testing.assert_array_equal(w.mask.cpu().numpy(), mask)
    assert resets > E  # teams were wiped out and envs restarted, several times
