set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05u; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_big.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_big.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_tdm_spill.py tests/test_gpu_tdm_wg.py tests/test_gpu_spill_wait.py tests/test_gpu_reward_sums.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit $?
for v in chunk lvlbig; do
  MACM_LIB=$PWD/abv/$v.so timeout -k 10 300 python bench.py --envs 256 --agents 2048 --steps 5 --warmup 2 --no-cpu-baseline > $O/big2048_$v.json 2> $O/big2048_$v.err || exit $?
  MACM_LIB=$PWD/abv/$v.so timeout -k 10 300 python bench.py --env tdm --teams 1024,1024 --envs 128 --steps 5 --warmup 2 --no-cpu-baseline > $O/tdmbig_$v.json 2> $O/tdmbig_$v.err || exit $?
  MACM_LIB=$PWD/abv/$v.so timeout -k 10 300 python bench.py --envs 64 --agents 4096 --steps 3 --warmup 2 --no-cpu-baseline > $O/big4096_$v.json 2> $O/big4096_$v.err || exit $?
done
echo ALLDONE
