#!/bin/bash
# Round 3: k_verify_r per host tile (SYDELTA_VERIFY_HALF=1) against per pair: its parity
# tests (scanner r), the C3 leg both ways; then scripts/r03y.sh (whole suite, smoke,
# default bench, rocprof trace + PMC).
set -u
TAG=${1:-r03z}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
SYDELTA_VERIFY_HALF=1 SYDELTA_TEST_SCANNERS=r timeout -k 10 400 python3 -u -m pytest tests/test_gpu_scan_large.py -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_half.log" 2>&1 || { tail -40 "$OUT/pytest_half.log"; exit 1; }
tail -1 "$OUT/pytest_half.log"
for h in 1 0; do
  SYDELTA_VERIFY_HALF=$h timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-inclusive \
    > "$OUT/half$h.json" 2> "$OUT/half$h.err" || { tail -20 "$OUT/half$h.err"; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/half$h.json').read().strip().splitlines()[-1]);print('half $h', d['value'], d['ms_per_step'], {k:v['avg_ms'] for k,v in d['kernels'].items() if 'scan' in k or 'verify' in k})"
done
bash scripts/r03y.sh r03y
