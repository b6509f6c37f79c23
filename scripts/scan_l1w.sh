#!/bin/bash
# First hardware run of k_scan_l1w (SYDELTA_SCAN_L1=2): large-index parity with the wide
# kernel in the parametrization, then phase timing at 1 GiB and the C3 bench line, each
# step under its own limit; stops at the first failure.
# Usage (from the repo root on the box): bash scripts/scan_l1w.sh [tag]
set -u
TAG=${1:-l1w}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
step() { local t=$1; shift; echo "== $* (limit ${t}s)" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== rc=$rc" >&2; return $rc; }
SYDELTA_TEST_SCAN_L1W=1 step 600 python -u -m pytest tests/test_gpu_scan_large.py -x -v -k l1w --timeout 300 \
  --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -4 "$OUT/pytest.log"
SYDELTA_SCAN_L1=2 SYDELTA_PHASE_TIMING=1 step 200 python bench.py --size-gib 1 --steps 2 --warmup 1 --no-cpu-baseline \
  --no-host-inclusive > "$OUT/timing.json" 2> "$OUT/timing.err" || { tail -20 "$OUT/timing.err"; exit 1; }
grep "phase cycles" "$OUT/timing.err" | tail -2
SYDELTA_SCAN_L1=2 step 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-inclusive \
  > "$OUT/bench_l1w.json" 2> "$OUT/bench_l1w.err" || { tail -20 "$OUT/bench_l1w.err"; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_l1w.json'));print('l1w', d['value'], d['ms_per_step'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"
step 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-inclusive \
  > "$OUT/bench_l1.json" 2> "$OUT/bench_l1.err" || { tail -20 "$OUT/bench_l1.err"; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_l1.json'));print('l1', d['value'], d['ms_per_step'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"
