#!/bin/bash
# Round-4 box session: instruction-cache counters of the metric window (is the wave kernel's code
# footprint a cost?). Lists the SQ / SQC counters first, then one PMC pass with the icache ones.
set -u
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
OUT=gpurun_out/${1:-r04ic}
mkdir -p "$OUT"
st() { echo "$1 rc=$2" | tee -a "$R/$OUT/status.txt"; [ "$2" -eq 0 ] || exit "$2"; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$R/$OUT/avail.txt" 2>&1; st list $?
grep -o "SQC_[A-Z0-9_]*\|SQ_IFETCH[A-Z0-9_]*\|SQ_WAIT_INST[A-Z0-9_]*\|SQ_INST_LEVEL[A-Z0-9_]*" "$R/$OUT/avail.txt" | sort -u > "$R/$OUT/icache_names.txt"
cat "$R/$OUT/icache_names.txt"
C=""
for c in SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH; do grep -qx "$c" "$R/$OUT/icache_names.txt" && C="$C $c"; done
echo "pass: $C" | tee -a "$R/$OUT/status.txt"
[ -n "$C" ] || exit 3
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv --pmc $C SQ_WAVES SQ_WAIT_INST_ANY -d "$R/$OUT/pmc_ic" -o run -- \
  python3 "$R/bench.py" --no-cpu-baseline --steps 20 --warmup 5 > "$R/$OUT/pmc_ic.json" 2> "$R/$OUT/pmc_ic.err"; st pmc_ic $?
echo ALLDONE | tee -a "$R/$OUT/status.txt"
