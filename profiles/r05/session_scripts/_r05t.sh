set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05t; mkdir -p $O
export MACM_STAMPS_LIB=$PWD/abv/stamps.so
timeout -k 10 300 python tools/big_phases.py --agents 2048 --envs 64 --warmup 2 --steps 3 --json $O/big2048.json > $O/big2048.log 2>&1 || exit $?
timeout -k 10 300 python tools/big_phases.py --agents 1500 --envs 64 --warmup 2 --steps 3 --json $O/big1500.json > $O/big1500.log 2>&1 || exit $?
echo ALLDONE
