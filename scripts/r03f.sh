#!/bin/bash
# Round 3: k_scan_l1 with the trimmed roll (bit-extract filter tests, constant LDS
# offsets, no partition code in the one-partition kernel, queue fast path): parity of
# every large-index and wide-window scan (the level-1 bit moved to q[0..4]), then the C3
# line with phase cycles, and the ablations.
set -u
TAG=${1:-r03f}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
step() { local t=$1; shift; echo "== $* (limit ${t}s)" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== rc=$rc" >&2; return $rc; }
step 900 python3 -u -m pytest tests/test_gpu_scan_large.py tests/test_gpu_scan_wide.py -x -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for ab in 0 1 2 7; do
  SYDELTA_ABLATE=$ab timeout -k 10 200 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-inclusive \
    > "$OUT/ab$ab.json" 2> "$OUT/ab$ab.err" || { tail -20 "$OUT/ab$ab.err"; exit 1; }
  SYDELTA_ABLATE=$ab SYDELTA_PHASE_TIMING=1 timeout -k 10 200 python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline \
    --no-host-inclusive > "$OUT/ab${ab}_phase.json" 2> "$OUT/ab${ab}_phase.err" || { tail -20 "$OUT/ab${ab}_phase.err"; exit 1; }
  python3 - "$OUT/ab$ab.json" "$ab" "$OUT/ab${ab}_phase.err" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ph = [l for l in open(sys.argv[3]) if "phase" in l]
print("ablate", sys.argv[2], "k_scan_l1", d["kernels"]["k_scan_l1"]["avg_ms"], "ms |", ph[-1].split("]")[-1].strip() if ph else "")
PY
done
echo "== done"
