set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r01_pmc2
timeout -k 10 300 python -m pytest tests/test_gpu_tdm.py -q -rf > gpurun_out/r01_pmc2/pytest_tdm.log 2>&1; rc=$?
echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
bash tools/pmc.sh gpurun_out/r01_pmc2/flock --steps 50 --warmup 10 && \
bash tools/pmc.sh gpurun_out/r01_pmc2/tdm --env tdm --steps 50 --warmup 10
