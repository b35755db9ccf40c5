set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05o; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_rollout.py -k "serialized or handoff" -x -v --timeout 500 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit $?
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVES SQ_INSTS_VALU -d "$GRAFT_REPO_ROOT/$O/sq_c5" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --envs 2048 --agents 1024 --steps 4 --warmup 2 > "$GRAFT_REPO_ROOT/$O/sq_c5.json" 2> "$GRAFT_REPO_ROOT/$O/sq_c5.err") || exit $?
echo ALLDONE
