set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
bash tools/gpu_check.sh r05g c5 c3 mbots c4 || exit $?
O=gpurun_out/r05g
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o c5 -- python3 bench.py --envs 2048 --agents 1024 --steps 10 --warmup 2 --no-cpu-baseline > $O/prof_c5.json 2> $O/prof_c5.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o c3 -- python3 bench.py --envs 4096 --agents 256 --flocks 4 --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_c3.json 2> $O/prof_c3.err || exit $?
echo ALLDONE
