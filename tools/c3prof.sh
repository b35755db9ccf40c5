set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/c3prof; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
MACM_STAMPS_LIB=$PWD/ab/stamps_head.so timeout -k 10 200 python tools/phase_profile.py --envs 4096 --agents 256 --flocks 4 --policy bots --warmup 200 --steps 10 --json $OUT/c3b.json > $OUT/c3b.log 2>&1 || exit $?
bash tools/kprof.sh c3prof/k ab/head.so -- --envs 4096 --agents 256 --flocks 4 --policy bots --steps 50 --warmup 250 > $OUT/kprof.log 2>&1 || exit $?
echo ALLDONE
