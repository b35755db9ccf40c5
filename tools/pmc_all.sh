#!/bin/bash
# All PMC passes of a round: Flock (random), TDM, Flock closed loop -> tools/pmc_summary.py
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash tools/pmc.sh gpurun_out/${PMC_OUT:-pmc}/flock --steps 50 --warmup 10 && \
bash tools/pmc.sh gpurun_out/${PMC_OUT:-pmc}/tdm --env tdm --steps 50 --warmup 10 && \
bash tools/pmc.sh gpurun_out/${PMC_OUT:-pmc}/flock_bots --policy bots --steps 50 --warmup 330
