#!/bin/bash
# Round-2 evidence with the rollout launch (bench.py --launch rollout, the default): GPU tests,
# smoke, bench lines per config, rocprofv3 kernel traces + stats, PMC passes of the rollout kernel.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
OUT=gpurun_out/${1:-final5}
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
st() { echo "$1 rc=$2" | tee -a "$R/$OUT/status.txt"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1; st pytest_gpu $?
timeout -k 10 180 python __graft_entry__.py smoke > "$OUT/smoke.log" 2>&1; st smoke $?
b() { local name=$1; shift; timeout -k 10 400 python bench.py "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"; st "$name" $?; }
b m_driver --gpus 1 --steps 20 --warmup 5
b m_default
b m_steady --steps 1000 --warmup 100 --no-cpu-baseline
b m_f64_driver --steps 20 --warmup 5 --obs-f64 --no-cpu-baseline
b c2_1024x64 --envs 1024 --steps 300 --warmup 30 --no-cpu-baseline
b c3_driver --envs 4096 --agents 256 --flocks 4 --steps 20 --warmup 5 --no-cpu-baseline
b c3_steady --envs 4096 --agents 256 --flocks 4 --steps 100 --warmup 50 --no-cpu-baseline
b c4_driver --env tdm --steps 20 --warmup 5
b c4_steady --env tdm --steps 1000 --warmup 100 --no-cpu-baseline
b c5_driver --envs 2048 --agents 1024 --steps 20 --warmup 5 --no-cpu-baseline
b m_bots --policy bots --steps 300 --warmup 300 --no-cpu-baseline
cd /tmp && export TMPDIR=/tmp
prof() { local name=$1; shift; timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof_$name" -o run -- python3 "$R/bench.py" --no-cpu-baseline "$@" > "$R/$OUT/prof_$name.json" 2> "$R/$OUT/prof_$name.err"; st "prof_$name" $?; }
prof m --steps 20 --warmup 5
prof m_steady --steps 1000 --warmup 100
prof c4 --env tdm --steps 20 --warmup 5
cd "$R"
timeout -k 10 600 bash tools/pmc.sh "$OUT/pmc_m" --steps 20 --warmup 5 > "$OUT/pmc_m.log" 2>&1; st pmc_m $?
timeout -k 10 600 bash tools/pmc.sh "$OUT/pmc_tdm" --env tdm --steps 20 --warmup 5 > "$OUT/pmc_tdm.log" 2>&1; st pmc_tdm $?
echo ALLDONE | tee -a "$R/$OUT/status.txt"
