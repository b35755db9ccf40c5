set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/mtr
MACM_STAMPS_LIB=$PWD/ab/stamps_head.so timeout -k 10 200 python tools/phase_profile.py --envs 4096 --agents 64 --warmup 5 --steps 20 --json gpurun_out/mtr/m_transient.json > gpurun_out/mtr/m_transient.log 2>&1 || exit $?
MACM_STAMPS_LIB=$PWD/ab/stamps_head.so timeout -k 10 200 python tools/phase_profile.py --envs 4096 --agents 64 --warmup 300 --steps 20 --json gpurun_out/mtr/m_steady.json > gpurun_out/mtr/m_steady.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/mtr/bench_w5.json 2>/dev/null || exit $?
timeout -k 10 200 python bench.py --steps 20 --warmup 300 --no-cpu-baseline > gpurun_out/mtr/bench_w300.json 2>/dev/null || exit $?
timeout -k 10 200 python bench.py --steps 500 --warmup 5 --no-cpu-baseline > gpurun_out/mtr/bench_500.json 2>/dev/null || exit $?
echo ALLDONE
