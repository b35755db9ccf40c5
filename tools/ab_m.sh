#!/bin/bash
# A/B of library variants on the wave-kernel configs: M transient (warmup 5, 20 steps, the
# driver's window), M steady (300 + 300), C2, TDM C4, Flock bots closed loop. tools/ab_m.sh OUT lib...
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
for r in 1 2; do
  for i in $(seq 0 $(($# - 1))); do
    lib=${@:$((i + 1)):1}
    export MACM_LIB="$PWD/$lib"
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/v${i}_r${r}_mtr.json" 2>/dev/null || exit $?
    timeout -k 10 120 python bench.py --steps 300 --warmup 300 --no-cpu-baseline > "$OUT/v${i}_r${r}_mss.json" 2>/dev/null || exit $?
    timeout -k 10 120 python bench.py --envs 1024 --steps 300 --warmup 30 --no-cpu-baseline > "$OUT/v${i}_r${r}_c2.json" 2>/dev/null || exit $?
    timeout -k 10 120 python bench.py --env tdm --steps 300 --warmup 30 --no-cpu-baseline > "$OUT/v${i}_r${r}_c4.json" 2>/dev/null || exit $?
    timeout -k 10 120 python bench.py --policy bots --steps 100 --warmup 300 --no-cpu-baseline > "$OUT/v${i}_r${r}_mbots.json" 2>/dev/null || exit $?
  done
done
python3 - "$OUT" "$@" <<'PY'
import json, sys, glob, collections
out, libs = sys.argv[1], sys.argv[2:]
res = collections.defaultdict(list)
for f in glob.glob(f"{out}/v*_r*_*.json"):
    n = f.split("/")[-1][:-5]
    v, r, c = n.split("_", 2)
    try:
        d = json.loads(open(f).read().strip().splitlines()[0])
        res[(c, int(v[1:]))].append(d["ms_per_step"] * 1e3)
    except Exception:
        pass
for c in ("mtr", "mss", "c2", "c4", "mbots"):
    print(c.ljust(6) + "".join(f"  v{i} {min(res[(c, i)]) if res[(c, i)] else float('nan'):8.2f} us" for i in range(len(libs))))
PY
echo ALLDONE
