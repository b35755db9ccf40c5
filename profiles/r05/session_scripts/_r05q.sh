set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05q; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_rollout.py -k "handoff" -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit $?
bash tools/env_ab.sh r05q/c5 MACM_HEAVY_B "0 64 128 256" --envs 2048 --agents 1024 --steps 10 --warmup 2 > $O/c5.txt 2>&1 || exit $?
echo ALLDONE
