set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05i; mkdir -p $O
bash tools/env_ab.sh r05i/c3 MACM_WG_SLICES "1 0" --envs 4096 --agents 256 --flocks 4 --steps 20 --warmup 5 > $O/c3.txt 2>&1 || exit $?
bash tools/env_ab.sh r05i/c3b MACM_WG_SLICES "1 0" --envs 4096 --agents 256 --flocks 4 --policy bots --steps 50 --warmup 200 > $O/c3b.txt 2>&1 || exit $?
echo ALLDONE
