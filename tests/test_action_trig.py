"""The action trig and observation atan2 the kernels compute themselves
(gym-macm_amd/csrc/macm_math.h), built for the host from the same source and compared
with Python's math.sin / math.cos / math.atan2 (glibc: what the reference's
mvmnt.py:113-116 / combat.py:147 and mvmnt.py:197 call).

The forces and melee-ray offsets are float32 values derived from sin/cos(angle) and
sin/cos(angle + pi/2). tools/trig_check.c enumerates every float32 angle |a| < 2^19 and
requires every derived float32 value to equal glibc's; macm_action_trig gets there with
a 17-entry table of glibc values (csrc/trig_fix.inc) at the inputs where its polynomial
would round differently. Host and device builds agree bit for bit (tools/trig_gpu_check.hip
prints the same digest on the GPU; profiles/r01/trig/)."""
import ctypes
import math
import os
import re
import struct
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "gym-macm_amd", "csrc")


def _build(tmp, src, out, extra):
    cmd = ["gcc", "-O2", "-ffp-contract=off", "-I", CSRC, "-I", os.path.join(REPO, "tools"),
           *extra, os.path.join(REPO, "tools", src), "-lm", "-o", out]
    subprocess.run(cmd, check=True, cwd=tmp)
    return out


@pytest.fixture(scope="module")
def shim(tmp_path_factory):
    d = tmp_path_factory.mktemp("trig")
    lib = ctypes.CDLL(_build(d, "trig_shim.c", str(d / "libtrig.so"), ["-shared", "-fPIC"]))
    lib.shim_sincos.argtypes = [ctypes.c_double, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
    lib.shim_action_trig.argtypes = [ctypes.c_float, ctypes.POINTER(ctypes.c_double)]
    lib.shim_action_trig_raw.argtypes = [ctypes.c_double, ctypes.POINTER(ctypes.c_double)]
    lib.shim_obs_atan2.argtypes = [ctypes.c_double, ctypes.c_double]
    lib.shim_obs_atan2.restype = ctypes.c_double
    return lib


def action_trig(lib, a):
    out = (ctypes.c_double * 4)()
    lib.shim_action_trig(a, out)
    return list(out)


def glibc4(a):
    x = float(np.float32(a))
    return [math.sin(x), math.cos(x), math.sin(x + math.pi / 2), math.cos(x + math.pi / 2)]


def table_angles():
    txt = open(os.path.join(CSRC, "trig_fix.inc")).read()
    return [float.fromhex(m) for m in re.findall(r"\{(-?0x[0-9a-fp.+-]+)f,", txt)]


def f32_forces(s0, c0, s1, c1):
    """The float32 quantities the step derives (csrc/flock_step_w64.hip actions block)."""
    out = []
    for k0 in (-1.0, 0.0, 1.0):
        for k1 in (-1.0, 0.0, 1.0):
            for cc in (1.0, 1.0 / math.sqrt(2.0)):
                for F in (20.0, 16.0):
                    out.append(np.float32((c0 * k0 + c1 * k1) * cc * F))
                    out.append(np.float32((s0 * k0 + s1 * k1) * cc * F))
    out += [np.float32(2.0 * c0), np.float32(2.0 * s0)]
    return np.array(out, np.float32)


def test_table_entries_are_glibc_values(shim):
    angles = table_angles()
    assert len(angles) == 17
    for a in angles:
        assert float(np.float32(a)) == a
        got = action_trig(shim, a)
        assert got == glibc4(a), f"angle {a!r}"


def test_table_entries_are_needed(shim):
    """Without the table these angles would give float32 forces / ray offsets that differ
    from the reference's (macm_action_trig_raw: the shared-reduction pair below |a| = 4,
    two macm_sincos beyond)."""
    for a in table_angles():
        out = (ctypes.c_double * 4)()
        shim.shim_action_trig_raw(a, out)
        raw = f32_forces(*list(out))
        ref = f32_forces(*glibc4(a))
        assert not np.array_equal(raw.view(np.uint32), ref.view(np.uint32)), f"angle {a!r}"


def test_random_angles_match_glibc(shim):
    rng = np.random.default_rng(7)
    angles = np.concatenate([rng.uniform(-math.pi, math.pi, 20000), rng.uniform(-600, 600, 2000),
                             [0.0, -0.0, math.pi, -math.pi, math.pi / 2, -math.pi / 2, 1e-30, -1e-30]])
    for a in angles.astype(np.float32):
        got = action_trig(shim, float(a))
        ref = glibc4(float(a))
        assert np.array_equal(f32_forces(*got).view(np.uint32), f32_forces(*ref).view(np.uint32)), float(a)
        # f64 values within 1 ulp of glibc
        for g, r in zip(got, ref):
            assert abs(struct.unpack("<q", struct.pack("<d", g))[0] - struct.unpack("<q", struct.pack("<d", r))[0]) <= 1 \
                or (g == 0.0 and r == 0.0)


def test_obs_atan2_within_one_ulp(shim):
    rng = np.random.default_rng(8)
    ys = rng.uniform(-40, 40, 20000).astype(np.float32)
    xs = rng.uniform(-40, 40, 20000).astype(np.float32)
    ys[:100] = 0.0
    xs[100:200] = 0.0
    for y, x in zip(ys.tolist(), xs.tolist()):
        g, r = shim.shim_obs_atan2(y, x), math.atan2(y, x)
        gi, ri = struct.unpack("<q", struct.pack("<d", g))[0], struct.unpack("<q", struct.pack("<d", r))[0]
        assert abs(gi - ri) <= 1 or g == r, (y, x, g, r)


def test_exhaustive_float32_angles(tmp_path):
    """Every float32 angle |a| < 2^19, both signs (2.45e9 inputs, ~35 s on 8 cores)."""
    exe = _build(tmp_path, "trig_check.c", str(tmp_path / "trig_check"), ["-fopenmp"])
    r = subprocess.run([exe], capture_output=True, text=True, timeout=1200)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "inputs whose float32 forces / ray offsets differ from glibc's: 0 (|x| <= pi+0.1: 0)" in r.stdout
    assert "inputs: 2449473536 float32 values" in r.stdout
