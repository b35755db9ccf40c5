set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05k; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_rollout.py -k "solve_pairs" -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit $?
MACM_WG_SLICES=2 bash tools/env_ab.sh r05k/c3s2 MACM_SOLVE_PAIR "0 1" --envs 4096 --agents 256 --flocks 4 --steps 20 --warmup 5 > $O/c3s2.txt 2>&1 || exit $?
MACM_WG_SLICES=3 bash tools/env_ab.sh r05k/c3s3 MACM_SOLVE_PAIR "0 1" --envs 4096 --agents 256 --flocks 4 --steps 20 --warmup 5 > $O/c3s3.txt 2>&1 || exit $?
MACM_WG_SLICES=3 bash tools/env_ab.sh r05k/c3b MACM_SOLVE_PAIR "0 1" --envs 4096 --agents 256 --flocks 4 --policy bots --steps 50 --warmup 200 > $O/c3b.txt 2>&1 || exit $?
echo ALLDONE
