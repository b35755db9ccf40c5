"""Loading helpers for the golden vectors under tests/golden/ (made by make_golden.py
from the reference's own env code)."""
import glob
import json
import os

import numpy as np

from gym_macm.settings import flockSettings, to_config

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _all():
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN_DIR, "*.npz")))


def names():
    """Flock goldens (mvmnt.py)."""
    return [n for n in _all() if not n.startswith("tdm_")]


def tdm_names():
    """TDM goldens (combat.py)."""
    return [n for n in _all() if n.startswith("tdm_")]


def tdm_config(g, obs_f64=True):
    from gym_macm._abi import tdm_config_from_defaults
    m = g["meta"]
    c = tdm_config_from_defaults()
    sizes = m["n_agents"]
    c.n_teams = len(sizes)
    for t in range(4):
        c.team_size[t] = sizes[t] if t < len(sizes) else 0
    c.n_agents = sum(sizes)
    c.obs_f64 = 1 if obs_f64 else 0
    st = m["settings"]
    assert (st["hz"], st["time_limit"], st["cooldown_atk"], st["cooldown_mov_penalty"]) == (
        c.hz, c.time_limit, c.cooldown_atk, c.cooldown_mov_penalty)
    assert (st["world_width"], st["world_height"]) == (c.world_width, c.world_height)
    return c


def load(name):
    z = np.load(os.path.join(GOLDEN_DIR, name + ".npz"), allow_pickle=False)
    g = {k: z[k] for k in z.files}
    g["meta"] = json.loads(str(g["meta"]))
    return g


def config(g, obs_f64=True):
    m = g["meta"]
    s = flockSettings(**m["kwargs"])
    return to_config(s, m["N"], m["T"], obs_f64=obs_f64), g["targets_idx"]


def wrap_diff(a, b):
    """Angular difference folded into [-pi, pi] (an ulp change at |t|=pi may flip the wrap)."""
    d = np.asarray(a, np.float64) - np.asarray(b, np.float64)
    return np.abs((d + np.pi) % (2 * np.pi) - np.pi)


def obs_close(obs, ref, od, rtol=4e-16, atol=1e-15):
    """Distances exact to a few f64 ulp; angles (atan2) to a few ulp modulo 2pi.
    numpy's arctan2 and glibc/ocml atan2 differ by <= 1 ulp (measured), which a
    subtraction of the body angle and one wrap can grow to a few ulp."""
    half = od // 2
    ok = True
    for base in (0, half):
        ok &= np.allclose(obs[..., base], ref[..., base], rtol=rtol, atol=atol)
        if od == 4:
            ok &= bool((wrap_diff(obs[..., base + 1], ref[..., base + 1]) <= 1e-14).all())
        else:
            ok &= np.allclose(obs[..., base + 1:base + 3], ref[..., base + 1:base + 3], rtol=0, atol=1e-14)
    return bool(ok)
