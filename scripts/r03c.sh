#!/bin/bash
# Round 3: first hardware run of the stripe-per-thread scan k_scan_s (SYDELTA_SCAN_L1=3 at
# the C3 shape, SYDELTA_SCAN_WIDE=2 for wide windows): its parity tests, then the C3 line
# and the bs-65536 line with it, against the defaults.  Each step under its own limit;
# stops at the first failure.
# Usage (from the repo root on the box): bash scripts/r03c.sh [tag]
set -u
TAG=${1:-r03c}
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
SYDELTA_TEST_SCANNERS=s step 900 python3 -u -m pytest tests/test_gpu_scan_large.py tests/test_gpu_scan_wide.py -x -v --timeout 300 \
  --timeout-method thread -p no:cacheprovider > "$OUT/pytest_s.log" 2>&1 || { tail -40 "$OUT/pytest_s.log"; exit 1; }
tail -4 "$OUT/pytest_s.log"
SYDELTA_SCAN_L1=3 leg c3_s --steps 10 --warmup 3 --no-cpu-baseline --no-host-inclusive || exit 1
leg c3_l1 --steps 10 --warmup 3 --no-cpu-baseline --no-host-inclusive || exit 1
SYDELTA_SCAN_WIDE=2 leg c3_bs64k_s --block-size 65536 --steps 3 --warmup 1 --no-cpu-baseline --no-host-inclusive || exit 1
leg c3_bs64k_w --block-size 65536 --steps 3 --warmup 1 --no-cpu-baseline --no-host-inclusive || exit 1
echo "== done"
