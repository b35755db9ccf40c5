set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05h; mkdir -p $O
export MACM_STAMPS_LIB=$PWD/abv/stamps.so
timeout -k 10 200 python tools/phase_profile.py --envs 2048 --agents 1024 --warmup 2 --steps 4 --json $O/c5.json > $O/c5.log 2>&1 || exit $?
timeout -k 10 200 python tools/phase_profile.py --envs 4096 --agents 256 --flocks 4 --warmup 5 --steps 10 --json $O/c3.json > $O/c3.log 2>&1 || exit $?
timeout -k 10 200 python tools/phase_profile.py --envs 4096 --agents 256 --flocks 4 --policy bots --warmup 200 --steps 10 --json $O/c3b.json > $O/c3b.log 2>&1 || exit $?
echo ALLDONE
