"""Device bots (csrc/bots.hip via macm_bots_*) vs the vectorised reference bots
(tests/parity.py, pinned to the reference's recorded bot actions), and closed-loop
rollouts `step -> device bot -> step` vs the oracle driven by the numpy bots.
Bar: identical actions (integer), bit-exact states."""
import numpy as np
import pytest
import torch

from oracle import OracleTDM
from parity import assert_state_equal, combat_bot, flock_bot, oracle_for

pytestmark = pytest.mark.gpu

from gym_macm.bots import combat_actions, flock_actions  # noqa: E402
from gym_macm.settings import flockSettings, to_config  # noqa: E402
from gym_macm.tdm_world import TdmWorld, tdm_config  # noqa: E402
from gym_macm.vec import FlockVec  # noqa: E402


def _edge_values(rng, shape):
    """Angles/distances with exact threshold and sign cases mixed in."""
    v = rng.uniform(-np.pi, np.pi, size=shape)
    special = np.array([0.0, -0.0, np.pi / 4, -np.pi / 4, np.pi / 5, -np.pi / 5, np.cos(np.pi / 4), 1.0, 3.0,
                        np.nextafter(np.pi / 4, 0), np.nextafter(1.0, 0), np.nextafter(3.0, 4)])
    pick = rng.random(shape) < 0.2
    v[pick] = rng.choice(special, size=int(pick.sum()))
    return v


@pytest.mark.parametrize("od", [4, 6])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_flock_bot_kernel_matches_reference_bot(od, dtype):
    rng = np.random.default_rng(od)
    obs = _edge_values(rng, (64, 33, od))
    obs[..., od // 2] = np.abs(rng.uniform(0, 2, size=(64, 33)))
    obs[rng.random((64, 33)) < 0.05, od // 2] = 1.0
    obs = obs.astype(dtype)
    a = flock_actions(torch.from_numpy(obs).cuda()).cpu().numpy()
    np.testing.assert_array_equal(a, flock_bot(obs.astype(np.float64)))


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_combat_bot_kernel_matches_reference_bot(dtype):
    rng = np.random.default_rng(1)
    E, N = 50, 17
    obs = _edge_values(rng, (E, N, N - 1, 4))
    obs[..., 0] = np.round(rng.uniform(0, 6, size=(E, N, N - 1)), 1)  # ties in r
    obs[..., 3] = rng.integers(0, 2, size=(E, N, N - 1))
    mask = (rng.random((E, N, N - 1)) < 0.8).astype(np.uint8)
    mask[0] = 0  # no enemies at all
    obs = obs.astype(dtype)
    a = combat_actions(torch.from_numpy(obs).cuda(), torch.from_numpy(mask).cuda()).cpu().numpy()
    np.testing.assert_array_equal(a, combat_bot(obs.astype(np.float64), mask))


def test_flock_closed_loop_on_device_bit_exact():
    """FlockVec(obs f64) + device bots.flock vs the oracle + the numpy bot."""
    E, N, seed = 16, 32, 21
    vec = FlockVec(E, n_agents=[N], seed=seed, device="cuda:0", obs_dtype=torch.float64, start_spread=10)
    orc = oracle_for(to_config(flockSettings(start_spread=10), N, 1, obs_f64=True), None, E, seed)
    obs, _ = orc.observe()
    act = torch.empty((E, N, 3), dtype=torch.uint8, device="cuda:0")
    for t in range(300):
        flock_actions(vec.obs, out=act)
        a = flock_bot(obs)
        np.testing.assert_array_equal(act.cpu().numpy(), a, err_msg=f"actions step {t}")
        vec.step(act)
        r = orc.step(a)
        obs = r["obs"]
        if t % 25 == 24:
            assert_state_equal(vec.get_state(), orc.get_state(vec.world.C), f"step {t}")
    assert int(vec.counters()[2]) > 0  # agents reach their targets


def test_tdm_closed_loop_on_device_bit_exact():
    E, teams, seed = 16, [8, 8], 4
    w = TdmWorld(tdm_config(teams, obs_f64=True, world_width=14.0, world_height=14.0), E, device="cuda:0")
    w.reset(seed)
    orc = OracleTDM(tdm_config(teams, obs_f64=True, world_width=14.0, world_height=14.0), E, seed)
    obs, mask = orc.observe()
    act = torch.empty((E, 16, 4), dtype=torch.uint8, device="cuda:0")
    for t in range(400):
        combat_actions(w.obs, w.mask, out=act)
        a = combat_bot(obs, mask)
        alive = orc.get_state()["alive"].astype(bool)
        np.testing.assert_array_equal(act.cpu().numpy()[alive], a[alive], err_msg=f"actions step {t}")
        w.step(act)
        r = orc.step(a)
        obs, mask = r["obs"], r["mask"]
        np.testing.assert_array_equal(w.health.cpu().numpy(), r["health"], err_msg=f"health step {t}")
    s = w.get_state()
    o = orc.get_state()
    for k in ("pos", "vel", "angle", "alive", "health", "winner", "done"):
        np.testing.assert_array_equal(s[k], o[k], err_msg=k)
    assert (s["winner"] >= 0).any()
