"""The CPU oracle's TDM env (oracle/tdm_oracle.c) against golden vectors made by
running the reference's own gym_macm/envs/combat.py (tests/golden/make_golden.py,
which supplies the four names combat.py needs but never defines; see
TDM_NOTE there and DESIGN.md "TDM").

Tolerances: positions, angles, health, cooldowns, alive, done, winner, listener:
exact. Observation: r, p and is_ally exact in f64 up to a few ulp; t (atan2) to a
few ulp modulo 2pi (numpy arctan2 vs glibc atan2)."""
import numpy as np
import pytest

import goldens
from oracle import OracleTDM


def tdm_obs_close(a, b, m):
    a = a[m.astype(bool)]
    b = b[m.astype(bool)]
    ok = np.allclose(a[:, 0], b[:, 0], rtol=4e-16, atol=1e-15)
    ok &= bool((goldens.wrap_diff(a[:, 1], b[:, 1]) <= 1e-14).all())
    ok &= bool((goldens.wrap_diff(a[:, 2], b[:, 2]) <= 1e-14).all())
    ok &= bool((a[:, 3] == b[:, 3]).all())
    return bool(ok)


@pytest.mark.parametrize("name", goldens.tdm_names())
def test_tdm_oracle_matches_reference_env(name):
    g = goldens.load(name)
    cfg = goldens.tdm_config(g)
    orc = OracleTDM(cfg, 1, g["meta"]["seed"])
    st = orc.get_state()
    np.testing.assert_array_equal(st["pos"][0], g["init_pos"])
    np.testing.assert_array_equal(st["angle"][0], g["init_angle"])
    obs0, mask0 = orc.observe()
    np.testing.assert_array_equal(mask0[0], g["init_mask"])
    assert tdm_obs_close(obs0[0], g["init_obs"], g["init_mask"])
    for t in range(g["meta"]["steps"]):
        r = orc.step(g["actions"][t][None])
        s = orc.get_state()
        np.testing.assert_array_equal(s["pos"][0], g["pos"][t], err_msg=f"pos step {t}")
        np.testing.assert_array_equal(s["angle"][0], g["angle"][t], err_msg=f"angle step {t}")
        np.testing.assert_array_equal(r["health"][0], g["health"][t], err_msg=f"health step {t}")
        np.testing.assert_array_equal(r["alive"][0], g["alive"][t], err_msg=f"alive step {t}")
        np.testing.assert_array_equal(s["cd_atk"][0], g["cd_atk"][t], err_msg=f"cd_atk step {t}")
        np.testing.assert_array_equal(s["cd_mov"][0], g["cd_mov"][t], err_msg=f"cd_mov step {t}")
        np.testing.assert_array_equal(s["listener"][0], g["listener"][t], err_msg=f"listener step {t}")
        assert bool(r["done"][0]) == bool(g["done"][t]), f"done step {t}"
        assert int(r["winner"][0]) == int(g["winner"][t]), f"winner step {t}"
        assert s["time_passed"][0] == g["time_passed"][t]
        np.testing.assert_array_equal(r["mask"][0], g["mask"][t], err_msg=f"mask step {t}")
        assert tdm_obs_close(r["obs"][0], g["obs"][t], g["mask"][t]), f"obs step {t}"


def test_tdm_goldens_exercise_the_semantics():
    """The fixtures cover hits, deaths, a winner and the stale listener."""
    hits = deaths = winners = stale = 0
    for name in goldens.tdm_names():
        g = goldens.load(name)
        hits += int((np.diff(g["health"], axis=0) < 0).sum())
        deaths += int((g["alive"][-1] == 0).sum())
        winners += int(g["winner"][-1] >= 0)
        stale += int((g["listener"][:, 0] == 1).sum())
    assert hits > 50 and deaths > 10 and winners >= 3 and stale > 0


def test_vectorised_combat_bot_matches_recorded_reference_actions():
    """tests/parity.combat_bot (the workload generator of the TDM parity tests)
    reproduces every action the reference's bots.combat chose in the goldens."""
    from parity import combat_bot
    n = 0
    for name in goldens.tdm_names():
        g = goldens.load(name)
        if g["meta"]["policy"] != "combat":
            continue
        obs = np.concatenate([g["init_obs"][None], g["obs"][:-1]])
        mask = np.concatenate([g["init_mask"][None], g["mask"][:-1]])
        alive = np.concatenate([np.ones((1, g["alive"].shape[1]), np.uint8), g["alive"][:-1]]) == 1
        a = combat_bot(obs, mask)
        np.testing.assert_array_equal(a[alive], g["actions"][alive], err_msg=name)
        n += int(alive.sum())
    assert n > 10000
