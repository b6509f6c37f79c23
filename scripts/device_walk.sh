#!/bin/bash
# First hardware run of the device walk (K5b, SYDELTA_DEVICE_WALK=1): its parity tests,
# then the C5 line with the host walk and with the device walk (host timings on stderr),
# then a kernel trace of the device-walk line; each step under its own limit, stops at
# the first failure.
# Usage (from the repo root on the box): bash scripts/device_walk.sh [tag]
set -u
TAG=${1:-dwalk}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
step() { local t=$1; shift; echo "== $* (limit ${t}s)" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== rc=$rc" >&2; return $rc; }
step 600 python -u -m pytest tests/test_gpu_device_walk.py -x -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -4 "$OUT/pytest.log"
summ() {
  python - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d["value"], d["ms_per_step"], "ms/step", {k: v["avg_ms"] for k, v in d["kernels"].items()})
PY
}
SYDELTA_HOST_TIMING=1 step 300 python bench.py --workload c5 --steps 10 --warmup 3 \
  > "$OUT/bench_c5_host.json" 2> "$OUT/bench_c5_host.err" || { tail -20 "$OUT/bench_c5_host.err"; exit 1; }
summ "$OUT/bench_c5_host.json" c5-host-walk
SYDELTA_HOST_TIMING=1 step 300 python bench.py --workload c5 --steps 10 --warmup 3 --device-walk \
  > "$OUT/bench_c5_dev.json" 2> "$OUT/bench_c5_dev.err" || { tail -20 "$OUT/bench_c5_dev.err"; exit 1; }
summ "$OUT/bench_c5_dev.json" c5-device-walk
grep "device walk" "$OUT/bench_c5_dev.err" | tail -3
step 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o c5dev -- python bench.py --workload c5 --steps 5 \
  --warmup 2 --device-walk > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
find "$OUT/prof" -name "*kernel_stats.csv" | head -1 | xargs -r head -30
