set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05m; mkdir -p $O
MACM_LIB=$PWD/abv/pdfs.so timeout -k 10 500 python -u -m pytest tests/test_gpu_wide_levels.py tests/test_gpu_headline.py tests/test_gpu_parity.py tests/test_gpu_tdm.py tests/test_gpu_islands.py tests/test_gpu_dense.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_pdfs.log 2>&1 || exit $?
bash tools/ab.sh r05m/mbots abv/base.so abv/pdfs.so -- --policy bots --steps 100 --warmup 300 > $O/mbots_ab.txt 2>&1 || exit $?
bash tools/ab.sh r05m/mwin abv/base.so abv/pdfs.so -- --steps 20 --warmup 5 > $O/mwin_ab.txt 2>&1 || exit $?
bash tools/ab.sh r05m/c2 abv/base.so abv/pdfs.so -- --envs 1024 --steps 100 --warmup 100 > $O/c2_ab.txt 2>&1 || exit $?
bash tools/ab.sh r05m/c4 abv/base.so abv/pdfs.so -- --env tdm --steps 20 --warmup 5 > $O/c4_ab.txt 2>&1 || exit $?
echo ALLDONE
