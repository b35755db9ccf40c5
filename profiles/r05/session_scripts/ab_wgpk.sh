set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/wgpk
MACM_LIB=$PWD/abv/wgpk.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/wgpk/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -20 gpurun_out/wgpk/pytest.log; exit 1; }
tail -3 gpurun_out/wgpk/pytest.log
bash tools/ab.sh wgpk/c5w abv/base.so abv/wgpk.so -- --envs 2048 --agents 1024 --steps 10 --warmup 2 && \
bash tools/ab.sh wgpk/c3w abv/base.so abv/wgpk.so -- --envs 4096 --agents 256 --flocks 4 --steps 20 --warmup 5
