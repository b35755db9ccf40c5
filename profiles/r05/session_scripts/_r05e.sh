set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05e; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_tdm_wg.py tests/test_gpu_reset.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit $?
MACM_HANDOFF=1 bash tools/env_ab.sh r05e/c5h MACM_FUSE_DFS "1 0" --envs 2048 --agents 1024 --steps 10 --warmup 2 > $O/c5h.txt 2>&1 || exit $?
MACM_HANDOFF=0 bash tools/env_ab.sh r05e/c5 MACM_FUSE_DFS "1 0" --envs 2048 --agents 1024 --steps 10 --warmup 2 > $O/c5.txt 2>&1 || exit $?
MACM_HANDOFF=1 bash tools/env_ab.sh r05e/c3h MACM_FUSE_DFS "1 0" --envs 4096 --agents 256 --flocks 4 --steps 20 --warmup 5 > $O/c3h.txt 2>&1 || exit $?
MACM_LIB=$PWD/abv/widepk.so timeout -k 10 300 python -u -m pytest tests/test_gpu_wide_levels.py tests/test_gpu_headline.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_widepk.log 2>&1 || exit $?
bash tools/ab.sh r05e/mbots_pk abv/base.so abv/widepk.so -- --policy bots --steps 100 --warmup 300 > $O/mbots_pk.txt 2>&1 || exit $?
bash tools/ab.sh r05e/mwin_pk abv/base.so abv/widepk.so -- --steps 20 --warmup 5 > $O/mwin_pk.txt 2>&1 || exit $?
echo ALLDONE
