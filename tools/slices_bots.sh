# sliced closed-loop workgroup rollout: rollout tests, C3 bots line (rollout_bots vs per-step launches)
set -u
mkdir -p gpurun_out/slb
timeout -k 10 300 python -u -m pytest tests/test_gpu_rollout.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/slb/pytest.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --envs 4096 --agents 256 --flocks 4 --policy bots --steps 100 --warmup 200 --no-cpu-baseline > gpurun_out/slb/c3_bots.json 2> gpurun_out/slb/c3_bots.err || exit 1
