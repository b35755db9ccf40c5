#!/bin/bash
# Per-kernel VGPRs and scratch bytes of the product TUs (compiler remarks), one line per kernel:
#   tools/kernel_resources.sh <dir holding csrc/>   (diff two trees to see what a change costs)
cd $1
for f in csrc/flock_step_w64.hip csrc/flock_rollout_w64.hip csrc/flock_step_wg.hip csrc/tdm_step_wg.hip; do
  extra=""; [ $f = csrc/flock_rollout_w64.hip ] && extra="-mllvm -disable-machine-licm"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize $extra -Rpass-analysis=kernel-resource-usage -c -o /dev/null $f 2>&1 | grep -E "Function Name|VGPRs:|ScratchSize" | paste - - - | sed -E 's/.*Function Name: ([^ ]*).*VGPRs: ([0-9]+).*lane\]: ([0-9]+).*/\1 \2 \3/' | sed "s#^#$(basename $f) #"
done
