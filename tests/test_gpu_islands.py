"""Island order of the workgroup path's islands-first DFS (kernel A, sparse worlds), bit-exact
against the CPU oracle's serial walk (b2World::Solve's DFS from the highest unvisited body).

The union-find must give every island the serial walk's seed (its highest body) and the islands
the serial walk's order (descending seeds). These layouts push it: a chain whose body indices
alternate high/low along it (labels hook in both directions and need several rounds), a star
(one body touching many), hundreds of two-body islands, a ring, and chains mixed with lone
bodies. Each runs 20 steps through the C-ABI with the oracle checked every step."""
import numpy as np
import pytest

from test_gpu_grid import inject, make_pair as make_pair_cells  # noqa: F401  (inject is shared)
import test_gpu_parity
from test_gpu_parity import check_rollout

pytestmark = pytest.mark.gpu


def run_layout(pos, seed, steps=20):
    E, N = pos.shape[:2]
    vec, orc = test_gpu_parity.make_pair(E, [N], seed=seed)
    inject(vec, orc, pos)
    rng = np.random.default_rng(seed)
    idle = lambda t: np.ones((E, N, 3), np.uint8) if t < 3 else rng.integers(0, 3, size=(E, N, 3)).astype(np.uint8)
    check_rollout(vec, orc, steps, rng, state_every=5, actions_fn=idle)


def far(N, k0):
    """positions 30 m apart on a far row for bodies k0..N-1 (no contacts)"""
    k = np.arange(N - k0)
    return np.stack([200.0 + 30.0 * (k % 40), -200.0 - 30.0 * (k // 40)], -1)


def test_zigzag_chain():
    """One chain of 120 bodies, spacing 0.95 (touching neighbours only), body ids along the chain
    0, 119, 1, 118, ...: every contact joins a low and a high id."""
    E, N = 2, 160
    ids = np.empty(120, int)
    ids[0::2] = np.arange(60)
    ids[1::2] = 119 - np.arange(60)
    pos = np.zeros((E, N, 2), np.float32)
    for e in range(E):
        pos[e, ids] = np.stack([np.arange(120) * 0.95 - 57.0, np.full(120, 3.0 * e)], -1)
        pos[e, 120:] = far(N, 120)
    run_layout(pos, seed=31)


def test_star_and_ring():
    """A star (body 7 with 6 touching neighbours on a circle of radius 0.98) and a ring of 40
    bodies (neighbours 0.96 apart), ids shuffled."""
    E, N = 2, 128
    rng = np.random.default_rng(2)
    pos = np.zeros((E, N, 2), np.float32)
    for e in range(E):
        perm = rng.permutation(N)
        star = [np.array([0.0, 0.0])] + [0.98 * np.array([np.cos(a), np.sin(a)]) for a in np.arange(6) * np.pi / 3]
        ang = np.arange(40) * 2 * np.pi / 40
        rr = 0.96 / (2 * np.sin(np.pi / 40))
        ring = np.stack([30.0 + rr * np.cos(ang), rr * np.sin(ang)], -1)
        pts = np.concatenate([np.array(star), ring, far(N, 47)])
        pos[e, perm] = pts
    run_layout(pos, seed=32)


def test_many_pairs():
    """128 two-body islands (touching pairs 0.9 apart, 5 m between pairs), ids shuffled: the
    most islands a 256-body env can have, ranked from 128 roots."""
    E, N = 2, 256
    rng = np.random.default_rng(3)
    pos = np.zeros((E, N, 2), np.float32)
    for e in range(E):
        k = np.arange(128)
        cen = np.stack([(k % 16) * 5.0 - 40.0, (k // 16) * 5.0 - 20.0], -1)
        pts = np.concatenate([cen, cen + np.array([0.9, 0.0])])
        pos[e, rng.permutation(N)] = pts
    run_layout(pos, seed=33)


def test_chains_and_loners():
    """20 chains of 6 bodies (ids random) between 80 lone bodies."""
    E, N = 2, 200
    rng = np.random.default_rng(4)
    pos = np.zeros((E, N, 2), np.float32)
    for e in range(E):
        chains = [np.stack([np.arange(6) * 0.97 + (c % 5) * 12.0, np.full(6, (c // 5) * 6.0)], -1) for c in range(20)]
        pts = np.concatenate(chains + [far(N, 120)])
        pos[e, rng.permutation(N)] = pts
    run_layout(pos, seed=34)
