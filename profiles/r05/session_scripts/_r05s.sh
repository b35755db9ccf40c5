set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05s; mkdir -p $O
MACM_LIB=$PWD/abv/pdfsw.so timeout -k 10 500 python -u -m pytest tests/test_gpu_wide_levels.py tests/test_gpu_headline.py tests/test_gpu_tdm_spill.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_pdfsw.log 2>&1 || exit $?
bash tools/ab.sh r05s/mbots abv/base.so abv/pdfsw.so -- --policy bots --steps 100 --warmup 300 > $O/mbots_ab.txt 2>&1 || exit $?
bash tools/ab.sh r05s/mwin abv/base.so abv/pdfsw.so -- --steps 20 --warmup 5 > $O/mwin_ab.txt 2>&1 || exit $?
echo ALLDONE
