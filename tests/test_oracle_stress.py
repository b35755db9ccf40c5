"""The CPU oracle on dense and large worlds (CPU suite, and the sanitizer leg: tools/asan_oracle.sh
runs this file against the -fsanitize=address,undefined build). The goldens are small (N <= 64);
these drive b2lite's growth paths — pair buffer, contact pool, edge lists, island stacks — at the
BASELINE sizes' densities: invariants of the contact list after every step, and two runs equal."""
import numpy as np
import pytest

from oracle import OracleFlock, OracleTDM
from gym_macm.settings import flockSettings, to_config
from gym_macm.tdm_world import tdm_config


def run_flock(N, spread, steps, E=2, seed=5):
    cfg = to_config(flockSettings(start_spread=spread), N, 1, obs_f64=True)
    orc = OracleFlock(cfg, None, E, seed)
    rng = np.random.default_rng(seed)
    for t in range(steps):
        r = orc.step(rng.integers(0, 3, size=(E, N, 3)).astype(np.uint8), n_threads=2)
        nbr = r["nbr_id"]
        assert ((nbr >= 0) & (nbr < N) & (nbr != np.arange(N)[None])).all(), f"step {t}"
    st = orc.get_state(N * (N - 1) // 2)
    for e in range(E):
        ab = st["contact_ab"][e, :int(st["contact_count"][e])].astype(np.int64)
        assert ((ab & 0xFFFF) < (ab >> 16)).all() and len(np.unique(ab)) == len(ab)
    return st


@pytest.mark.parametrize("N,spread,steps", [(64, 3, 20), (256, 8, 6), (1024, 14, 2)])
def test_dense_flock_worlds(N, spread, steps):
    a = run_flock(N, spread, steps)
    b = run_flock(N, spread, steps)
    for k in ("pos", "vel", "contact_count"):
        np.testing.assert_array_equal(a[k], b[k])


def test_dense_tdm_world():
    orc = OracleTDM(tdm_config([12, 12], obs_f64=True, world_width=6.0, world_height=6.0), 2, 9)
    rng = np.random.default_rng(9)
    for _ in range(40):
        a = rng.integers(0, 3, size=(2, 24, 4)).astype(np.uint8)
        a[..., 3] = rng.integers(0, 2, size=(2, 24))
        orc.step(a)
    st = orc.get_state()
    assert ((st["health"] * 4) == np.round(st["health"] * 4)).all()
