set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05r; mkdir -p $O
export MACM_STAMPS_LIB=$PWD/abv/stamps.so
timeout -k 10 200 python tools/phase_profile.py --envs 4096 --agents 64 --warmup 5 --steps 20 --json $O/mwin.json > $O/mwin.log 2>&1 || exit $?
timeout -k 10 200 python tools/phase_profile.py --envs 4096 --agents 64 --warmup 100 --steps 20 --json $O/msteady.json > $O/msteady.log 2>&1 || exit $?
echo ALLDONE
