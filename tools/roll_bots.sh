# closed-loop rollout: tests, then M / C4 bots lines (rollout_bots vs per-step launches in the same run)
set -u
mkdir -p gpurun_out/rbots
timeout -k 10 300 python -u -m pytest tests/test_gpu_rollout.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/rbots/pytest.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --policy bots --steps 300 --warmup 300 --no-cpu-baseline > gpurun_out/rbots/m_bots.json 2> gpurun_out/rbots/m_bots.err || exit 1
timeout -k 10 300 python bench.py --env tdm --policy bots --steps 300 --warmup 30 --no-cpu-baseline > gpurun_out/rbots/c4_bots.json 2> gpurun_out/rbots/c4_bots.err || exit 1
timeout -k 10 300 python bench.py --policy bots --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/rbots/m_bots_window.json 2> gpurun_out/rbots/m_bots_window.err || exit 1
