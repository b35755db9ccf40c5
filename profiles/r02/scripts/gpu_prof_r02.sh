#!/bin/bash
# rocprofv3 kernel traces/stats and PMC passes of the final tree (rollout launch, the default)
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-final8}
mkdir -p "$R/$OUT"
st() { echo "$1 rc=$2" | tee -a "$R/$OUT/status.txt"; [ "$2" -eq 0 ] || exit "$2"; }
cd /tmp && export TMPDIR=/tmp
prof() { local name=$1; shift; timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof_$name" -o run -- python3 "$R/bench.py" --no-cpu-baseline "$@" > "$R/$OUT/prof_$name.json" 2> "$R/$OUT/prof_$name.err"; st "prof_$name" $?; }
prof m --steps 20 --warmup 5
prof m_steady --steps 1000 --warmup 100
prof c4 --env tdm --steps 20 --warmup 5
prof m_bots --policy bots --steps 300 --warmup 300
cd "$R"
timeout -k 10 600 bash tools/pmc.sh "$OUT/pmc_m" --steps 20 --warmup 5 > "$OUT/pmc_m.log" 2>&1; st pmc_m $?
timeout -k 10 600 bash tools/pmc.sh "$OUT/pmc_tdm" --env tdm --steps 20 --warmup 5 > "$OUT/pmc_tdm.log" 2>&1; st pmc_tdm $?
echo ALLDONE | tee -a "$R/$OUT/status.txt"
