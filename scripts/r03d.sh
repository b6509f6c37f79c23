#!/bin/bash
# Round 3: k_scan_l1 with deferred verification (SYDELTA_SCAN_DEFER=1: passes listed,
# k_pass_verify looks them up and verifies them afterwards): parity, phase cycles, C3 A/B.
# Usage (from the repo root on the box): bash scripts/r03d.sh [tag]
set -u
TAG=${1:-r03d}
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
print(sys.argv[2], d["value"], d["unit"], d["ms_per_step"], "ms/step", r.get("kernel"), r.get("frac"),
      {k: (v["avg_ms"], v["launches"]) for k, v in (d.get("kernels") or {}).items()}, d.get("match_stats"))
PY
}
leg() { local name=$1; shift; step 400 python3 -u bench.py "$@" > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err" \
  || { tail -20 "$OUT/bench_$name.err"; return 1; }; summ "$OUT/bench_$name.json" "$name"; }
SYDELTA_TEST_SCANNERS=${SCANNERS:-l1d} step 900 python3 -u -m pytest tests/test_gpu_scan_large.py -x -v --timeout 300 \
  --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
SYDELTA_SCAN_DEFER=1 SYDELTA_PHASE_TIMING=1 step 200 python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline \
  --no-host-inclusive > "$OUT/phase.json" 2> "$OUT/phase.err" || { tail -20 "$OUT/phase.err"; exit 1; }
grep "phase" "$OUT/phase.err" | tail -1
SYDELTA_SCAN_DEFER=1 leg c3_defer --steps 10 --warmup 3 --no-cpu-baseline --no-host-inclusive || exit 1
leg c3_l1 --steps 10 --warmup 3 --no-cpu-baseline --no-host-inclusive || exit 1
echo "== done"
