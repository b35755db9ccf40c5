"""The workgroup path's spatial hash (csrc/flock_grid.hpp) against the CPU oracle's all-pairs
scans, through the C-ABI, bit-exact (same bar as test_gpu_parity.py).

The strip cells must give the reference's results for every layout (mvmnt.py:185-196 nearest
neighbour, lowest index on ties; Box2D's pair set for the contact list). The cells are the
default sweep from N = 512; these tests force them at every N (DEBUG_SWEEP_CELLS) and push each
branch: nearest neighbours outside the wave's tile (the walk over the other strips), converged
clusters far apart, positions far from the origin (strip width raised to keep strip
coordinates small), exact distance ties on an integer lattice, fat AABBs far wider than the
others, and long dense rollouts of the C3 / C5 shapes."""
import numpy as np
import pytest
import torch

import test_gpu_parity
from test_gpu_parity import check_rollout, rand_actions

pytestmark = pytest.mark.gpu

from gym_macm import _abi  # noqa: E402


def make_pair(*a, **kw):
    """test_gpu_parity.make_pair with the strip-cell sweep forced on the HIP world."""
    vec, orc = test_gpu_parity.make_pair(*a, **kw)
    vec.world.set_debug(_abi.DEBUG_SWEEP_CELLS)
    return vec, orc


def inject(vec, orc, pos, fat_fn=None):
    """Place bodies at pos [E, N, 2] (zero velocity, fresh fat AABBs — or fat_fn(e, fat) — and
    the pair list of the overlapping fat AABBs in FindNewContacts order) in both worlds."""
    E, N = pos.shape[:2]
    C = vec.world.C
    # one step first: the oracle's first Step runs the pending FindNewContacts of the freshly
    # created fixtures (Box2D's e_newFixture), which would rebuild the injected fat AABBs
    idle = np.ones((E, N, 3), np.uint8)
    orc.step(idle)
    vec.step(torch.from_numpy(idle).cuda())
    st = orc.get_state(C)
    for e in range(E):
        p = pos[e].astype(np.float32)
        st["pos"][e] = p
        st["vel"][e] = 0.0
        st["sleep"][e] = 0.0
        st["fat"][e] = np.concatenate([(p - np.float32(0.5)) - np.float32(0.1),
                                       (p + np.float32(0.5)) + np.float32(0.1)], -1)
        if fat_fn is not None:
            fat_fn(e, st["fat"][e])
        f = st["fat"][e]
        lo, hi = f[:, :2], f[:, 2:]
        ov = ~((lo[None, :, 0] > hi[:, None, 0]) | (lo[None, :, 1] > hi[:, None, 1]) |
               (lo[:, None, 0] > hi[None, :, 0]) | (lo[:, None, 1] > hi[None, :, 1]))
        pairs = [(a, b) for a in range(N - 1, -1, -1) for b in np.nonzero(ov[a, a + 1:])[0][::-1] + a + 1]
        assert len(pairs) <= C
        st["contact_count"][e] = len(pairs)
        st["contact_ab"][e] = 0
        if pairs:
            st["contact_ab"][e, :len(pairs)] = [a | (int(b) << 16) for a, b in pairs]
        st["contact_imp"][e] = 0.0
    orc.set_state(st)
    vec.set_state(st)


def test_sparse_world_neighbours_beyond_the_tile():
    """start_spread 300: nearest neighbours ~25 m away, many strips: agents whose neighbour lies
    outside their wave's tile take the walk over the other strips."""
    vec, orc = make_pair(4, [128], seed=21, start_spread=300)
    check_rollout(vec, orc, 40, np.random.default_rng(21), state_every=10)


def test_converged_clusters_far_apart():
    """Four tight flocks of 64 (spacing 1.05: many touching pairs) 120 m apart plus four lone
    agents between them: clustered cells sharing buckets, lone agents' neighbours in another
    flock."""
    E, N = 2, 260
    vec, orc = make_pair(E, [N], seed=5, targets=[min(i // 64, 3) for i in range(N)])
    rng = np.random.default_rng(8)
    pos = np.zeros((E, N, 2), np.float32)
    for e in range(E):
        for f, (ox, oy) in enumerate([(-60, -60), (60, -60), (-60, 60), (60, 60)]):
            k = np.arange(64)
            pos[e, 64 * f:64 * f + 64] = np.stack([ox + (k % 8) * 1.05, oy + (k // 8) * 1.05], -1)
        pos[e, 256:] = rng.uniform(-40, 40, size=(4, 2))
        pos[e] += rng.uniform(-0.01, 0.01, size=(N, 2)).astype(np.float32)
    inject(vec, orc, pos)
    check_rollout(vec, orc, 40, rng, state_every=10)


def test_far_from_origin_raises_cell_side():
    """A 20 m flock 1e5 m from the origin (float32 spacing ~0.008 m there): strip coordinates
    are taken relative to the env's smallest x."""
    vec, orc = make_pair(3, [200], seed=9, start_spread=20, start_point=[1.0e5, -7.5e4])
    check_rollout(vec, orc, 30, np.random.default_rng(9), state_every=10)


def test_integer_lattice_exact_ties():
    """Agents on an integer lattice of spacing 2 (exactly representable, not touching): every
    agent has 2-4 neighbours at exactly the same squared distance; the lowest index must win,
    whatever order the hash visits them in. Agent ids are shuffled over the lattice."""
    E, N = 2, 144
    vec, orc = make_pair(E, [N], seed=3)
    rng = np.random.default_rng(4)
    k = np.arange(N)
    lat = np.stack([(k % 12) * 2.0 - 11.0, (k // 12) * 2.0 - 11.0], -1).astype(np.float32)
    pos = np.stack([lat[rng.permutation(N)] for _ in range(E)])
    inject(vec, orc, pos)
    vec.observe()
    o0, n0 = orc.observe()
    np.testing.assert_array_equal(vec.nbr_id.cpu().numpy(), n0)
    # no-op actions keep the lattice (and the ties) for the first steps
    check_rollout(vec, orc, 20, rng, state_every=5,
                  actions_fn=lambda t: np.ones((E, N, 3), np.uint8) if t < 10 else rand_actions(rng, E, N))


def test_c5_dense_1024_agents_long():
    """BASELINE config 5 shape, 2 envs x 60 steps: the dense start relaxes past the reset
    transient (one giant island, then separating and sleeping islands)."""
    vec, orc = make_pair(2, [1024], seed=56)
    check_rollout(vec, orc, 60, np.random.default_rng(56), state_every=20)


def test_c3_converging_flocks():
    """BASELINE config 3 (256 agents, 4 targets) with every agent pushed toward its flock's
    target each step (the bots' heading, not random walks): the flocks contract into dense
    clusters over 120 steps."""
    E, N = 2, 256
    tg = [i // 64 for i in range(N)]
    vec, orc = make_pair(E, [N], seed=77, targets=tg)
    rng = np.random.default_rng(77)

    def toward(t):
        # observation-driven policy: rotate toward the target angle (polar obs [.., 3]), push
        # forward; a few random agents per step keep the contact set changing
        obs = vec.obs.cpu().numpy()
        ang = obs[..., 3]
        a = np.ones((E, N, 3), np.uint8)
        a[..., 0] = np.where(ang > 0.1, 2, np.where(ang < -0.1, 0, 1))
        a[..., 1] = 2
        m = rng.random((E, N)) < 0.05
        a[m] = rand_actions(rng, E, N)[m]
        return a

    check_rollout(vec, orc, 120, rng, state_every=20, actions_fn=toward)


def test_big_fat_aabbs():
    """Bodies whose fat AABBs are far wider than the others' (a body that drifted inside an old
    fat box, or a fast one): 2 m, 6 m and 300 m boxes widen every tile (Dx) and are kept while
    they contain their bodies."""
    E, N = 2, 200
    vec, orc = make_pair(E, [N], seed=12, max_contacts=20000)
    rng = np.random.default_rng(12)
    pos = rng.uniform(-9, 9, size=(E, N, 2)).astype(np.float32)

    def widen(e, f):
        for k, (w, h) in zip((3, 50, 77 + e, 150), ((2.0, 1.3), (6.0, 6.0), (300.0, 300.0), (1.3, 4.0))):
            c = pos[e, k]
            f[k] = np.array([c[0] - w / 2, c[1] - h / 2, c[0] + w / 2, c[1] + h / 2], np.float32)

    inject(vec, orc, pos, widen)
    check_rollout(vec, orc, 30, rng, state_every=5)


@pytest.mark.parametrize("flag", [_abi.DEBUG_SWEEP_ALL_PAIRS, 0])
def test_c5_sweep_modes_agree(flag):
    """C5 shape with the all-pairs sweep forced, and with the default (strip cells at 1024)."""
    vec, orc = test_gpu_parity.make_pair(2, [1024], seed=57)
    vec.world.set_debug(flag)
    check_rollout(vec, orc, 20, np.random.default_rng(57), state_every=10)
