set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05j; mkdir -p $O
bash tools/env_ab.sh r05j/c3q4 MACM_WG_SLICES "2 3 4" --envs 4096 --agents 256 --flocks 4 --steps 20 --warmup 5 > $O/c3q4.txt 2>&1 || exit $?
GPU_MAX_HW_QUEUES=8 bash tools/env_ab.sh r05j/c3q8 MACM_WG_SLICES "2 3 4 6" --envs 4096 --agents 256 --flocks 4 --steps 20 --warmup 5 > $O/c3q8.txt 2>&1 || exit $?
echo ALLDONE
