set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05v; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_tdm_wg.py tests/test_gpu_tdm_spill.py tests/test_gpu_spill_wait.py tests/test_gpu_big.py tests/test_gpu_tdm.py tests/test_gpu_reward_sums.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit $?
for v in lvlall; do
  MACM_LIB=$PWD/abv/$v.so timeout -k 10 300 python bench.py --env tdm --teams 64,64 --envs 1024 --steps 20 --warmup 5 --no-cpu-baseline > $O/tdm128_$v.json 2> $O/tdm128_$v.err || exit $?
  MACM_LIB=$PWD/abv/$v.so timeout -k 10 300 python bench.py --env tdm --teams 256,256 --envs 256 --steps 10 --warmup 3 --no-cpu-baseline > $O/tdm512_$v.json 2> $O/tdm512_$v.err || exit $?
  MACM_LIB=$PWD/abv/$v.so timeout -k 10 300 python bench.py --env tdm --steps 20 --warmup 5 --no-cpu-baseline > $O/c4_$v.json 2> $O/c4_$v.err || exit $?
done
echo ALLDONE
