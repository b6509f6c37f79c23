#!/bin/bash
# Every bench workload once, one JSON line per leg under gpurun_out/<tag>/, each leg
# under its own time limit; stops at the first failing leg.
# Usage (from the repo root on the box): bash scripts/bench_legs.sh [tag] [legs...]
#   default legs: c3 c3b c2 c5 c4 path apply json local xxh3 (sigjson and zstd: first hardware runs, named explicitly)
set -u
TAG=${1:-legs}; shift || true
LEGS=${*:-c3 c3b c2 c5 c4 path apply json local xxh3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
for w in $LEGS; do
  echo "== $w" >&2
  timeout -k 10 400 python -u bench.py --workload "$w" > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err"
  rc=$?
  if [ $rc -ne 0 ]; then echo "== $w rc=$rc" >&2; tail -20 "$OUT/bench_$w.err"; exit 1; fi
  python - "$OUT/bench_$w.json" "$w" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline") or {}
print(sys.argv[2], d["value"], d["unit"], d["ms_per_step"], "ms/step", r.get("kernel"), r.get("frac"),
      {k: v["avg_ms"] for k, v in (d.get("kernels") or {}).items()},
      "cpu", (d.get("cpu_baseline") or {}).get("value"), "host_incl", d.get("host_inclusive"))
PY
done
echo "== done"
