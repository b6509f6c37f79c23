#!/bin/bash
# Round 3: k_scan_l2 (SYDELTA_SCAN_L1=4: k_scan_l1 on 32 Ki-position tiles, 112 KiB
# level-1 filter) with one or two batches of level-2 loads in flight
# (SYDELTA_SCAN_DEPTH): parity, phase cycles, C3 A/B against k_scan_l1.
set -u
TAG=${1:-r03g}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
step() { local t=$1; shift; echo "== $* (limit ${t}s)" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== rc=$rc" >&2; return $rc; }
SYDELTA_TEST_SCANNERS=l2 step 600 python3 -u -m pytest tests/test_gpu_scan_large.py -x -v --timeout 300 \
  --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for cfg in 4:2 4:1 1:1; do
  m=${cfg%%:*}; export SYDELTA_SCAN_DEPTH=${cfg##*:}
  SYDELTA_SCAN_L1=$m timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-inclusive \
    > "$OUT/m$cfg.json" 2> "$OUT/m$cfg.err" || { tail -20 "$OUT/m$cfg.err"; exit 1; }
  SYDELTA_SCAN_L1=$m SYDELTA_PHASE_TIMING=1 timeout -k 10 200 python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline \
    --no-host-inclusive > "$OUT/m${cfg}_phase.json" 2> "$OUT/m${cfg}_phase.err" || { tail -20 "$OUT/m${cfg}_phase.err"; exit 1; }
  python3 - "$OUT/m$cfg.json" "$cfg" "$OUT/m${cfg}_phase.err" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ph = [l for l in open(sys.argv[3]) if "phase" in l]
print("mode", sys.argv[2], d["value"], d["ms_per_step"], {k: v["avg_ms"] for k, v in d["kernels"].items()}, "|", ph[-1].split("]")[-1].strip() if ph else "")
PY
done
echo "== done"
