"""The C-ABI library loads on a machine without a GPU, exports exactly what
include/macm.h declares, and fails (without aborting) when no device exists."""
import ctypes
import os
import re

import pytest

from gym_macm import _abi

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "macm.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(macm_[a-z_]+)\s*\(", src)))


def test_header_declares_the_abi():
    fns = declared_functions()
    assert "macm_world_step" in fns and "macm_world_create" in fns
    assert set(fns) == set(_abi.SIGNATURES), "ctypes mirror out of sync with include/macm.h"


def test_library_exports_every_declared_symbol():
    L = _abi.lib()
    for name in declared_functions():
        assert hasattr(L, name), name


def test_struct_layouts_match_header():
    # sizes fixed by the header's field order (no implicit padding surprises)
    assert ctypes.sizeof(_abi.MacmConfig) == 10 * 4 + 10 * 8 + 4 * 4
    assert ctypes.sizeof(_abi.MacmOutputs) == 5 * 8
    assert ctypes.sizeof(_abi.MacmState) == 11 * 8
    assert ctypes.sizeof(_abi.MacmWorldInfo) == 8 * 4
    assert ctypes.sizeof(_abi.MacmTdmConfig) == 12 * 4 + 12 * 8 + 4 * 4
    assert ctypes.sizeof(_abi.MacmTdmOutputs) == 6 * 8
    assert ctypes.sizeof(_abi.MacmTdmState) == 17 * 8


def test_tdm_defaults_match_python_mirror():
    L = _abi.lib()
    c = _abi.MacmTdmConfig()
    assert L.macm_tdm_config_default(ctypes.byref(c)) == 0
    assert bytes(c) == bytes(_abi.tdm_config_from_defaults())
    c.team_size[0] = 40
    c.team_size[1] = 40
    c.n_agents = 80
    h = ctypes.c_void_p()
    assert L.macm_tdm_create(ctypes.byref(c), 4, 0, ctypes.byref(h)) == -4
    c.n_agents = 79
    assert L.macm_tdm_create(ctypes.byref(c), 4, 0, ctypes.byref(h)) == -1


def test_version_and_defaults_without_gpu():
    L = _abi.lib()
    assert L.macm_abi_version() == 2
    assert b"gfx950" in L.macm_version()
    c = _abi.MacmConfig()
    assert L.macm_config_default(ctypes.byref(c)) == 0
    assert (c.velocity_iterations, c.position_iterations, c.hz) == (8, 3, 60.0)
    assert c.radius == 0.5 and abs(c.agent_rotation_speed - 0.8 * 2 * 3.141592653589793) == 0


def test_invalid_config_is_rejected_with_message():
    L = _abi.lib()
    c = _abi.MacmConfig()
    L.macm_config_default(ctypes.byref(c))
    c.n_agents = 1
    h = ctypes.c_void_p()
    rc = L.macm_world_create(ctypes.byref(c), None, 4, 0, 0, ctypes.byref(h))
    assert rc == -1 and b"n_agents" in L.macm_last_error()
    c.n_agents = 1025
    assert L.macm_world_create(ctypes.byref(c), None, 4, 0, 0, ctypes.byref(h)) == -4


@pytest.mark.skipif(os.environ.get("HIP_VISIBLE_DEVICES") is None and os.path.exists("/dev/kfd"),
                    reason="only meaningful where no GPU is visible")
def test_no_device_returns_error_not_abort():
    L = _abi.lib()
    c = _abi.MacmConfig()
    L.macm_config_default(ctypes.byref(c))
    h = ctypes.c_void_p()
    rc = L.macm_world_create(ctypes.byref(c), None, 4, 0, 0, ctypes.byref(h))
    assert rc in (-1, -3)
    assert L.macm_last_error()


def test_header_is_plain_c():
    import subprocess
    r = subprocess.run(["gcc", "-x", "c", "-std=c99", "-Wall", "-Werror", "-fsyntax-only", HEADER],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
