set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05w; mkdir -p $O
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/m_driver.json 2> $O/m_driver.err || exit $?
timeout -k 10 400 python bench.py --env tdm --steps 20 --warmup 5 --no-cpu-baseline > $O/c4_window.json 2> $O/c4.err || exit $?
bash tools/configs_r05.sh r05w/configs > $O/configs.txt 2>&1 || exit $?
echo ALLDONE
