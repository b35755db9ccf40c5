set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05f; mkdir -p $O
for v in pklv pkch; do
  MACM_LIB=$PWD/abv/$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_parity.py tests/test_gpu_wide_levels.py tests/test_gpu_tdm.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_$v.log 2>&1 || exit $?
done
bash tools/ab.sh r05f/mwin abv/base.so abv/pklv.so abv/pkch.so -- --steps 20 --warmup 5 > $O/mwin.txt 2>&1 || exit $?
bash tools/ab.sh r05f/mbots abv/base.so abv/pklv.so abv/pkch.so -- --policy bots --steps 100 --warmup 300 > $O/mbots.txt 2>&1 || exit $?
bash tools/ab.sh r05f/c2 abv/base.so abv/pklv.so abv/pkch.so -- --envs 1024 --steps 100 --warmup 100 > $O/c2.txt 2>&1 || exit $?
bash tools/ab.sh r05f/c4 abv/base.so abv/pkch.so -- --env tdm --steps 20 --warmup 5 > $O/c4.txt 2>&1 || exit $?
echo ALLDONE
