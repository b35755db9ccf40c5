set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/tail2
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider tests/test_gpu_tdm_split.py -k tail > gpurun_out/tail2/pytest_tail.log 2>&1 || { echo "tail tests failed"; exit 1; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider tests/test_gpu_tdm.py tests/test_gpu_tdm_split.py tests/test_gpu_trajectory.py tests/test_gpu_tdm_spill.py tests/test_gpu_headline.py > gpurun_out/tail2/pytest_tdm.log 2>&1 || { echo "tdm tests failed"; exit 1; }
bash tools/tail_ab.sh tail2/ab
