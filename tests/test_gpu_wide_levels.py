"""Gauss-Seidel levels of the wave kernel beyond 64 touching contacts (round 3), bit-exact against
the CPU oracle's serial Box2D solve (b2Island::Solve over the DFS order).

The wave kernel (N <= 64) solves an env level by level once an island has more than 4 contacts.
Up to round 2 that needed T <= 64 touching contacts (one per lane); converged flocks have islands
of 60-100 contacts (the reference's bots.flock closed loop, test_scripts/bots.py:37-61), which one
lane then walked serially. Now contact k sits in slot k / 64 of lane k % 64: two slots up to 128
contacts (scalar DFS), four up to 256 (lane-0 DFS). These layouts reach every slot count:

  * square 8 x 8 lattice, spacing 0.98: one island of 112 contacts (two slots)
  * square 8 x 8 lattice, spacing 0.70 (diagonals touch too): 210 contacts (four slots)
  * hexagonal 8 x 8 patch, spacing 0.98: 161 contacts (four slots)
  * a 6 x 6 hexagonal patch beside 14 touching pairs: 85 + 14 contacts in 15 islands
  * the bots.flock closed loop at 64 agents after 300 steps (converged flocks, T up to ~95)

Every step's rewards, neighbour ids and collision flags and, every few steps, the whole state
(positions, velocities, fat AABBs, sleep clocks, the ordered contact list with its impulses) must
equal the oracle's."""
import numpy as np
import pytest
import torch

from parity import assert_state_equal, flock_bot, oracle_for
from test_gpu_grid import inject
import test_gpu_parity
from test_gpu_parity import check_rollout

pytestmark = pytest.mark.gpu

from gym_macm.bots import flock_actions  # noqa: E402
from gym_macm.settings import flockSettings, to_config  # noqa: E402
from gym_macm.vec import FlockVec  # noqa: E402


def touching(pos, ab, cnt):
    a, b = ab[:cnt] & 0xFFFF, ab[:cnt] >> 16
    d = pos[b] - pos[a]
    return int(((d * d).sum(-1) <= np.float32(1.0)).sum())


def square(n, h):
    k = np.arange(n * n)
    return np.stack([(k % n) * h, (k // n) * h], -1)


def hexagon(nx, ny, h):
    k = np.arange(nx * ny)
    r, c = k // nx, k % nx
    return np.stack([c * h + (r % 2) * h / 2, r * h * np.sqrt(3) / 2], -1)


def run_layout(pts, seed, steps=40, t_min=65):
    """pts [E, 64, 2]: ids shuffled per env; idle for 3 steps, then random actions"""
    E, N = pts.shape[:2]
    vec, orc = test_gpu_parity.make_pair(E, [N], seed=seed)
    rng = np.random.default_rng(seed)
    pos = np.zeros((E, N, 2), np.float32)
    for e in range(E):
        pos[e, rng.permutation(N)] = pts[e] + np.float32(7.0 * e)
    inject(vec, orc, pos)
    st = orc.get_state(vec.world.C)
    T = [touching(st["pos"][e], st["contact_ab"][e], st["contact_count"][e]) for e in range(E)]
    assert min(T) >= t_min, f"layout has too few touching contacts: {T}"
    idle = lambda t: np.ones((E, N, 3), np.uint8) if t < 3 else rng.integers(0, 3, size=(E, N, 3)).astype(np.uint8)
    check_rollout(vec, orc, steps, rng, state_every=2, actions_fn=idle)
    assert vec.spilled() == 0, "the layout went to the spill step instead of the wave kernel's levels"
    return T


def test_square_lattice_two_slots():
    pts = np.stack([square(8, 0.98) for _ in range(3)]).astype(np.float32)
    T = run_layout(pts, seed=51)
    assert max(T) <= 128


def test_square_lattice_diagonals_four_slots():
    pts = np.stack([square(8, 0.70) for _ in range(3)]).astype(np.float32)
    T = run_layout(pts, seed=52, t_min=129)
    assert max(T) <= 256


def test_hex_patch_four_slots():
    pts = np.stack([hexagon(8, 8, 0.98) for _ in range(3)]).astype(np.float32)
    run_layout(pts, seed=53, t_min=129)


def test_hex_patch_beside_pairs():
    pairs = np.concatenate([np.stack([np.arange(14) * 3.0 + 10.0, np.full(14, -6.0)], -1),
                            np.stack([np.arange(14) * 3.0 + 10.9, np.full(14, -6.0)], -1)])
    pts = np.stack([np.concatenate([hexagon(6, 6, 0.98), pairs]) for _ in range(3)]).astype(np.float32)
    run_layout(pts, seed=54, steps=30)


def test_bots_closed_loop_64_agents_converged():
    """The metric config's agent count in the reference's bots.flock closed loop, 300 steps from
    reset (float64 obs, so the device bot decides on the reference's values): the flocks converge
    on their targets into islands of 60-100 contacts; checked through the whole approach."""
    E, N, seed = 32, 64, 0x6D61636D
    vec = FlockVec(E, n_agents=[N], seed=seed, device="cuda:0", obs_dtype=torch.float64)
    orc = oracle_for(to_config(flockSettings(), N, 1, obs_f64=True), None, E, seed)
    obs, _ = orc.observe()
    act = torch.empty((E, N, 3), dtype=torch.uint8, device="cuda:0")
    tmax = 0
    for t in range(300):
        flock_actions(vec.obs, out=act)
        a = flock_bot(obs)
        np.testing.assert_array_equal(act.cpu().numpy(), a, err_msg=f"actions step {t}")
        _, nbr, rew, _ = vec.step(act)
        r = orc.step(a, n_threads=8)
        obs = r["obs"]
        np.testing.assert_array_equal(rew.cpu().numpy(), r["reward"].astype(np.float32), err_msg=f"reward step {t}")
        np.testing.assert_array_equal(nbr.cpu().numpy(), r["nbr_id"], err_msg=f"nbr step {t}")
        if t % 20 == 19 or t >= 280:
            st = orc.get_state(vec.world.C)
            assert_state_equal(vec.get_state(), st, f"step {t}")
            tmax = max(tmax, max(touching(st["pos"][e], st["contact_ab"][e], st["contact_count"][e])
                                 for e in range(E)))
    assert vec.status() == 0
    assert tmax > 64, f"the closed loop never passed 64 touching contacts (max {tmax})"
