#!/bin/bash
# Round 3: k_scan_r with the lookups and verification deferred to k_verify_r: its
# large-index parity tests, then the C3 bench leg (mode 5 vs k_scan_l2) and the scan
# without drains (ablate 1) for reference.
set -u
TAG=${1:-r03s}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
SYDELTA_TEST_SCANNERS=r timeout -k 10 400 python3 -u -m pytest tests/test_gpu_scan_large.py -x -v \
  --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
for m in 5 4; do
  SYDELTA_SCAN_L1=$m timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-inclusive \
    > "$OUT/mode$m.json" 2> "$OUT/mode$m.err" || { tail -20 "$OUT/mode$m.err"; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/mode$m.json').read().strip().splitlines()[-1]);print('mode $m', d['value'], d['ms_per_step'], {k:v['avg_ms'] for k,v in d['kernels'].items()}, d.get('match_stats'))"
done
SYDELTA_SCAN_L1=5 SYDELTA_ABLATE=1 timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline \
  --no-host-inclusive > "$OUT/ab1.json" 2> "$OUT/ab1.err" || { tail -20 "$OUT/ab1.err"; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/ab1.json').read().strip().splitlines()[-1]);print('mode 5 ablate 1', {k:v['avg_ms'] for k,v in d['kernels'].items()})"
echo "== done"
