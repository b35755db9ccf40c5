# round 6 session: parity of the per-lane env-scalar variant, then its A/B against the shipped library
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/s2
MACM_LIB=$PWD/abv/scal_lane.so timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_reward_sums.py tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_dense.py tests/test_gpu_rollout.py tests/test_gpu_fullsize.py tests/test_gpu_tdm.py tests/test_gpu_tdm_split.py tests/test_gpu_tdm_spill.py tests/test_gpu_bots.py tests/test_gpu_reset.py tests/test_gpu_trajectory.py > gpurun_out/s2/pytest_scal.log 2>&1 || { echo "scal tests failed"; exit 1; }
bash tools/ab_m.sh s2/ab_scal abv/rsum_bin.so abv/cnt_lane.so abv/scal_lane.so
