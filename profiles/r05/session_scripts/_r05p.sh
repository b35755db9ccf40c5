set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05p; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_rollout.py tests/test_gpu_trajectory.py tests/test_gpu_bots.py tests/test_gpu_fullsize.py -k "closed or bots" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit $?
bash tools/ab.sh r05p/c3b abv/chunk.so abv/botc.so -- --envs 4096 --agents 256 --flocks 4 --policy bots --steps 50 --warmup 200 > $O/c3b.txt 2>&1 || exit $?
echo ALLDONE
