# sliced workgroup rollout: tests, C3 lines (window, steady), C5 window
set -u
mkdir -p gpurun_out/slc
timeout -k 10 300 python -u -m pytest tests/test_gpu_rollout.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/slc/pytest.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --envs 4096 --agents 256 --flocks 4 --steps 20 --warmup 5 > gpurun_out/slc/c3_driver.json 2> gpurun_out/slc/c3_driver.err || exit 1
timeout -k 10 300 python bench.py --envs 4096 --agents 256 --flocks 4 --steps 100 --warmup 50 --no-cpu-baseline > gpurun_out/slc/c3_steady.json 2> gpurun_out/slc/c3_steady.err || exit 1
timeout -k 10 300 python bench.py --envs 2048 --agents 1024 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/slc/c5_driver.json 2> gpurun_out/slc/c5_driver.err || exit 1
