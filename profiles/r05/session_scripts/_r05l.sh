set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05l; mkdir -p $O
export MACM_STAMPS_LIB=$PWD/abv/stamps.so
timeout -k 10 200 python tools/phase_profile.py --envs 2048 --agents 1024 --warmup 2 --steps 10 --json $O/c5.json > $O/c5.log 2>&1 || exit $?
timeout -k 10 200 python tools/phase_profile.py --envs 4096 --agents 256 --flocks 4 --warmup 5 --steps 20 --json $O/c3.json > $O/c3.log 2>&1 || exit $?
timeout -k 10 300 python tools/phase_profile.py --envs 4096 --agents 64 --policy bots --warmup 300 --steps 20 --json $O/mbots.json > $O/mbots.log 2>&1 || exit $?
unset MACM_STAMPS_LIB
bash tools/env_ab.sh r05l/c3b MACM_WG_SLICES "2 3" --envs 4096 --agents 256 --flocks 4 --policy bots --steps 50 --warmup 200 > $O/c3b.txt 2>&1 || exit $?
MACM_LIB=$PWD/abv/regmin.so timeout -k 10 300 python -u -m pytest tests/test_gpu_wide_levels.py tests/test_gpu_headline.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_regmin.log 2>&1 || exit $?
bash tools/ab.sh r05l/mbots abv/base.so abv/regmin.so -- --policy bots --steps 100 --warmup 300 > $O/mbots_ab.txt 2>&1 || exit $?
bash tools/ab.sh r05l/mwin abv/base.so abv/regmin.so -- --steps 20 --warmup 5 > $O/mwin_ab.txt 2>&1 || exit $?
echo ALLDONE
