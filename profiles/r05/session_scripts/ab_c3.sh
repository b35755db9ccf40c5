set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/ab.sh c3chk/c3w abv/base.so gym-macm_amd/libmacm_hip.so -- --envs 4096 --agents 256 --flocks 4 --steps 20 --warmup 5 && \
timeout -k 10 300 python bench.py --envs 4096 --agents 256 --flocks 4 --steps 20 --warmup 5 > gpurun_out/c3chk/c3_window_cpu.json 2> gpurun_out/c3chk/c3_window_cpu.err
