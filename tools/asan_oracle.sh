#!/bin/bash
# Sanitizer leg of the CPU oracle: build oracle/ with -fsanitize=address,undefined
# and run the oracle's own test suite (known-answer physics, every reference golden replay, TDM
# goldens) against it. Host code only, in this container (never on the GPU box).
#   tools/asan_oracle.sh [extra pytest flags]   # runs tests/test_oracle_*.py (ORACLE_TESTS overrides)
set -euo pipefail
REPO="$(cd "$(dirname "$0")/.." && pwd)"
make -s -C "$REPO/oracle" asan
export MACM_ORACLE_LIB="$REPO/oracle/_asan/liboracle_flock.so"
# python is not instrumented: the ASan runtime must be the first library loaded; CPython's own
# allocations at exit are not the oracle's, so leak detection is off
export ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1"
export UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1"
export OMP_NUM_THREADS="${OMP_NUM_THREADS:-4}"
cd "$REPO"
TESTS=${ORACLE_TESTS:-tests/test_oracle_physics.py tests/test_oracle_golden.py tests/test_oracle_tdm_golden.py tests/test_oracle_stress.py}
# shellcheck disable=SC2086
LD_PRELOAD="$(gcc -print-file-name=libasan.so)" python -m pytest -q -p no:cacheprovider "$@" $TESTS
