"""The CPU oracle's env layer (oracle/flock_oracle.c) against golden vectors made
by running the reference's own gym_macm/envs/mvmnt.py (tests/golden/make_golden.py).

Tolerances: positions, angles, neighbour ids, rewards, done: exact. Observation
values: a few f64 ulp (numpy arctan2 vs glibc atan2 differ by <= 1 ulp), and exact
after rounding to float32 except where noted."""
import numpy as np
import pytest

import goldens
from oracle import OracleFlock


@pytest.mark.parametrize("name", goldens.names())
def test_oracle_matches_reference_env(name):
    g = goldens.load(name)
    cfg, tidx = goldens.config(g)
    orc = OracleFlock(cfg, tidx, 1, g["meta"]["seed"])
    st = orc.get_state(max_contacts=cfg.n_agents * (cfg.n_agents - 1) // 2)
    np.testing.assert_array_equal(st["targets"][0], g["targets"])
    np.testing.assert_array_equal(st["pos"][0], g["init_pos"])
    np.testing.assert_array_equal(st["angle"][0], g["init_angle"])
    obs0, nbr0 = orc.observe()
    np.testing.assert_array_equal(nbr0[0], g["init_nbr"])
    assert goldens.obs_close(obs0[0], g["init_obs"], obs0.shape[-1])
    for t in range(g["meta"]["steps"]):
        r = orc.step(g["actions"][t][None])
        s = orc.get_state(max_contacts=cfg.n_agents * (cfg.n_agents - 1) // 2)
        np.testing.assert_array_equal(s["pos"][0], g["pos"][t], err_msg=f"pos step {t}")
        np.testing.assert_array_equal(s["angle"][0], g["angle"][t], err_msg=f"angle step {t}")
        np.testing.assert_array_equal(r["nbr_id"][0], g["nbr"][t], err_msg=f"nbr step {t}")
        np.testing.assert_array_equal(r["reward"][0], g["reward"][t], err_msg=f"reward step {t}")
        assert bool(r["done"][0]) == bool(g["done"][t]), f"done step {t}"
        assert goldens.obs_close(r["obs"][0], g["obs"][t], r["obs"].shape[-1]), f"obs step {t}"
        # collided agents are exactly the reward dict's -1 keys
        np.testing.assert_array_equal(r["collided"][0].astype(bool), g["reward"][t] == -1)


def test_golden_obs_f32_exact():
    """Rounded to float32 (the HIP path's default obs dtype) the oracle's f64 obs
    equal the reference's on every golden step checked here."""
    bad = 0
    total = 0
    for name in goldens.names():
        g = goldens.load(name)
        cfg, tidx = goldens.config(g)
        orc = OracleFlock(cfg, tidx, 1, g["meta"]["seed"])
        for t in range(min(g["meta"]["steps"], 100)):
            r = orc.step(g["actions"][t][None])
            a = r["obs"][0].astype(np.float32)
            b = g["obs"][t].astype(np.float32)
            bad += int((a != b).sum())
            total += a.size
    assert bad <= total * 1e-5, (bad, total)


def test_vectorised_flock_bot_matches_recorded_reference_actions():
    """tests/parity.flock_bot (the model of the device bots.flock kernel) reproduces
    every action the reference's bots.flock chose in the goldens."""
    from parity import flock_bot
    n = 0
    for name in goldens.names():
        g = goldens.load(name)
        if g["meta"]["policy"] != "bots":
            continue
        obs = np.concatenate([g["init_obs"][None], g["obs"][:-1]])
        np.testing.assert_array_equal(flock_bot(obs), g["actions"], err_msg=name)
        n += g["actions"].shape[0] * g["actions"].shape[1]
    assert n > 5000


@pytest.mark.parametrize("name", goldens.names())
def test_reward_dict_order_matches_reference(name):
    """The rewards dict's key order (mvmnt.py:160-179: world.contacts' fixture A then B, then the rest in
    ascending id) as the reference produced it (golden `reward_order`), two ways:
    - the oracle's own world list (b2lite's m_contactList order, fo_contacts) gives it directly;
    - the drop-in's reconstruction (gym_macm.envs.mvmnt.reward_key_order) from the ordered per-env lists
      the product keeps (the oracle's export of the same layout, before and after each step) gives it too.
    """
    from gym_macm.envs.mvmnt import reward_key_order
    g = goldens.load(name)
    cfg, tidx = goldens.config(g)
    N = cfg.n_agents
    C = N * (N - 1) // 2
    orc = OracleFlock(cfg, tidx, 1, g["meta"]["seed"])
    prev = orc.get_state(C)
    prev_ab = prev["contact_ab"][0, :prev["contact_count"][0]].copy()
    for t in range(g["meta"]["steps"]):
        orc.step(g["actions"][t][None])
        want = [int(x) for x in g["reward_order"][t]]
        world = dict()
        for a, b, _touching in orc.contacts(0):
            world.setdefault(int(a), None)
            world.setdefault(int(b), None)
        direct = list(world) + [i for i in range(N) if i not in world]
        assert direct == want, f"oracle world list order, step {t}"
        s = orc.get_state(C)
        nxt = s["contact_ab"][0, :s["contact_count"][0]].copy()
        keys, n_contact = reward_key_order(prev_ab, nxt, N)
        assert keys == want, f"reconstructed order, step {t}"
        assert n_contact == int((g["reward"][t] == -1).sum())
        prev_ab = nxt
