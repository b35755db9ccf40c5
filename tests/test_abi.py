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


def test_struct_layouts_match_header(tmp_path):
    """Every field offset and struct size of the ctypes mirror equals what a C compiler lays
    out from include/macm.h (gcc, no GPU needed)."""
    import subprocess
    structs = {"macm_config": _abi.MacmConfig, "macm_outputs": _abi.MacmOutputs, "macm_state": _abi.MacmState,
               "macm_world_info": _abi.MacmWorldInfo, "macm_tdm_config": _abi.MacmTdmConfig,
               "macm_tdm_outputs": _abi.MacmTdmOutputs, "macm_tdm_state": _abi.MacmTdmState}
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void) {"]
    for cname, cls in structs.items():
        lines.append(f'  printf("{cname} %zu\\n", sizeof({cname}));')
        for f, _ in cls._fields_:
            lines.append(f'  printf("{cname}.{f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("  return 0;\n}")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    r = subprocess.run(["gcc", "-std=c99", "-o", str(exe), str(src)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    got = dict(line.rsplit(" ", 1) for line in subprocess.run([str(exe)], capture_output=True, text=True,
                                                               check=True).stdout.split("\n") if line)
    for cname, cls in structs.items():
        assert int(got[cname]) == ctypes.sizeof(cls), cname
        for f, _ in cls._fields_:
            assert int(got[f"{cname}.{f}"]) == getattr(cls, f).offset, f"{cname}.{f}"


def test_tdm_defaults_match_python_mirror():
    L = _abi.lib()
    c = _abi.MacmTdmConfig()
    assert L.macm_tdm_config_default(ctypes.byref(c)) == 0
    assert bytes(c) == bytes(_abi.tdm_config_from_defaults())
    c.team_size[0] = 2049  # above the workgroup step's 4096 agents: refused before any HIP call
    c.team_size[1] = 2048
    c.n_agents = 4097
    h = ctypes.c_void_p()
    assert L.macm_tdm_create(ctypes.byref(c), 4, 0, ctypes.byref(h)) == -4
    c.n_agents = 4096
    assert L.macm_tdm_create(ctypes.byref(c), 4, 0, ctypes.byref(h)) == -1


def test_version_and_defaults_without_gpu():
    L = _abi.lib()
    assert L.macm_abi_version() == 9
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
    c.n_agents = 4097  # above 4 bodies per thread of a 1024-thread workgroup (flock_big.hip)
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
