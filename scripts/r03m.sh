#!/bin/bash
# Round 3: the §8f rows' bench legs on this round's tree (sigjson, dparse, zstd -- their
# first bench run on hardware -- apply, json, local, xxh3), the bs-65536 legs with their
# CPU baselines, and the rocprof kernel trace of the bs-65536 C3 command.  Each step under
# its own limit; stops at the first failure.
set -u
TAG=${1:-r03m}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
step() { local t=$1; shift; echo "== $* (limit ${t}s)" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== rc=$rc" >&2; return $rc; }
summ() {
  python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline") or {}
c = d.get("cpu_baseline") or {}
print(sys.argv[2], d["value"], d["unit"], d["ms_per_step"], "ms/step", r.get("kernel"), r.get("frac"),
      {k: (v["avg_ms"], v["launches"]) for k, v in (d.get("kernels") or {}).items()}, "cpu", c.get("value"), c.get("unit"))
PY
}
leg() { local name=$1; shift; step 400 python3 -u bench.py "$@" > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err" \
  || { tail -20 "$OUT/bench_$name.err"; return 1; }; summ "$OUT/bench_$name.json" "$name"; }
for w in sigjson dparse zstd apply json local xxh3; do leg "$w" --workload "$w" || exit 1; done
leg c3_bs64k --block-size 65536 --steps 5 --warmup 2 --no-host-inclusive || exit 1
leg c5_bs64k_4g --workload c5 --block-size 65536 --size-gib 4 --steps 5 --warmup 2 || exit 1
cd /tmp
step 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_bs64k" -o run --output-format csv -- python3 "$R/bench.py" \
  --block-size 65536 --steps 5 --warmup 2 --no-cpu-baseline --no-host-inclusive > "$OUT/prof_bs64k.log" 2>&1 \
  || { tail -20 "$OUT/prof_bs64k.log"; exit 1; }
head -6 "$OUT"/trace_bs64k/*/run_kernel_stats.csv 2>/dev/null || find "$OUT/trace_bs64k" -name "*kernel_stats.csv" -exec head -6 {} \;
echo "== done"
