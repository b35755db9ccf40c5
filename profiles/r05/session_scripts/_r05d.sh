set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_grid.py tests/test_gpu_islands.py tests/test_gpu_fullsize.py tests/test_gpu_dense.py tests/test_gpu_reward_sums.py tests/test_gpu_rollout.py tests/test_gpu_trajectory.py tests/test_gpu_wide_levels.py tests/test_gpu_spill_wait.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || exit $?
bash tools/env_ab.sh r05d/c5 MACM_HANDOFF "1 0" --envs 2048 --agents 1024 --steps 10 --warmup 2 > $O/c5.txt 2>&1 || exit $?
bash tools/env_ab.sh r05d/c3s MACM_HANDOFF "1 0" --envs 1000 --agents 256 --flocks 4 --steps 20 --warmup 5 > $O/c3small.txt 2>&1 || exit $?
bash tools/solo_ab.sh r05d/mbots "0 32 128" --policy bots --steps 100 --warmup 300 > $O/mbots.txt 2>&1 || exit $?
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/m_driver.json 2> $O/m_driver.err || exit $?
echo ALLDONE
