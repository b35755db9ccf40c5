set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/s1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_reward_sums.py tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_dense.py tests/test_gpu_rollout.py tests/test_gpu_fullsize.py > gpurun_out/s1/pytest_rsum.log 2>&1 || { echo "rsum tests failed"; exit 1; }
MACM_LIB=$PWD/abv/rsum_rb2.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_tdm.py tests/test_gpu_tdm_split.py tests/test_gpu_tdm_spill.py tests/test_gpu_bots.py > gpurun_out/s1/pytest_rb2.log 2>&1 || { echo "rb2 tests failed"; exit 1; }
bash tools/ab_m.sh s1/ab_rsum abv/cur.so abv/rsum_bin.so && bash tools/ab_c4.sh s1/ab_rb2 abv/rsum_bin.so abv/rsum_rb2.so
