"""The sanitizer leg of SURVEY.md §5: the CPU oracle (the parity checker of every GPU test) built with
-fsanitize=address,undefined (make -C oracle asan) and its own tests run against that build
(tools/asan_oracle.sh: known-answer physics, every reference golden replay, TDM goldens, dense and
1024-agent worlds). Host code only; it runs here in the CPU suite, never on the GPU box."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(600)
def test_oracle_suite_under_asan_and_ubsan():
    gcc = shutil.which("gcc")
    if gcc is None or not os.path.exists(subprocess.run([gcc, "-print-file-name=libasan.so"], capture_output=True,
                                                        text=True).stdout.strip()):
        pytest.skip("no gcc ASan runtime")
    p = subprocess.run([os.path.join(REPO, "tools", "asan_oracle.sh")], capture_output=True, text=True, timeout=580)
    assert p.returncode == 0, (p.stdout[-3000:], p.stderr[-3000:])
    assert " passed" in p.stdout and "error" not in p.stderr.lower(), p.stderr[-3000:]
