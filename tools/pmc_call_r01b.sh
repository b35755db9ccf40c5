set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash tools/pmc.sh gpurun_out/r01_pmc3/flock --steps 50 --warmup 10 && \
bash tools/pmc.sh gpurun_out/r01_pmc3/tdm --env tdm --steps 50 --warmup 10 && \
bash tools/pmc.sh gpurun_out/r01_pmc3/flock_bots --policy bots --steps 50 --warmup 330
