set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05n; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_big.py tests/test_gpu_dense.py tests/test_gpu_tdm_spill.py tests/test_gpu_tdm_wg.py tests/test_gpu_spill_wait.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit $?
for v in base chunk; do
  MACM_LIB=$PWD/abv/$v.so timeout -k 10 300 python bench.py --envs 256 --agents 2048 --steps 5 --warmup 2 --no-cpu-baseline > $O/big2048_$v.json 2> $O/big2048_$v.err || exit $?
  MACM_LIB=$PWD/abv/$v.so timeout -k 10 300 python bench.py --env tdm --teams 1024,1024 --envs 128 --steps 5 --warmup 2 --no-cpu-baseline > $O/tdmbig_$v.json 2> $O/tdmbig_$v.err || exit $?
  MACM_LIB=$PWD/abv/$v.so timeout -k 10 300 python bench.py --envs 2048 --agents 1024 --steps 10 --warmup 2 --no-cpu-baseline > $O/c5_$v.json 2> $O/c5_$v.err || exit $?
done
echo ALLDONE
