#!/bin/bash
# Round 3: k_scan_w on 32 Ki-position tiles with k_scan_l2's trimmed roll -- its parity
# tests (k_scan_w only), then the bs-65536 legs (5 % byte edits: every position
# literal; C5-style 1 % block edits) and the kernel's phase cycles.  Each step under its
# own limit; stops at the first failure.
set -u
TAG=${1:-r03k}
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
SYDELTA_TEST_SCANNERS=w step 600 python3 -u -m pytest tests/test_gpu_scan_wide.py tests/test_gpu_stream_path.py -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_w.log" 2>&1 || { tail -40 "$OUT/pytest_w.log"; exit 1; }
tail -2 "$OUT/pytest_w.log"
leg c3_bs64k --block-size 65536 --steps 5 --warmup 2 --no-cpu-baseline --no-host-inclusive || exit 1
leg c5_bs64k_4g --workload c5 --block-size 65536 --size-gib 4 --steps 5 --warmup 2 --no-cpu-baseline || exit 1
SYDELTA_PHASE_TIMING=1 step 200 python3 bench.py --block-size 65536 --steps 1 --warmup 1 --no-cpu-baseline \
  --no-host-inclusive > "$OUT/phase_bs64k.json" 2> "$OUT/phase_bs64k.err" || { tail -20 "$OUT/phase_bs64k.err"; exit 1; }
grep -i "phase\|cycles" "$OUT/phase_bs64k.err" | tail -5
echo "== done"
