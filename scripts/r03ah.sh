#!/bin/bash
# Round 3: k_scan_r with the verification inline (SYDELTA_SCAN_R_INLINE=1: lookups at each
# wave tile's end, windows hashed from the registers): its large-index parity tests, then
# the C3 leg both ways.
set -u
TAG=${1:-r03ah}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
SYDELTA_SCAN_R_INLINE=1 SYDELTA_TEST_SCANNERS=r timeout -k 10 400 python3 -u -m pytest tests/test_gpu_scan_large.py -x -v \
  --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for i in 1 0; do
  SYDELTA_SCAN_R_INLINE=$i timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-inclusive \
    > "$OUT/inline$i.json" 2> "$OUT/inline$i.err" || { tail -20 "$OUT/inline$i.err"; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/inline$i.json').read().strip().splitlines()[-1]);print('inline $i', d['value'], d['ms_per_step'], {k:v['avg_ms'] for k,v in d['kernels'].items() if 'scan' in k or 'verify' in k}, d['match_stats'])"
done
echo "== done"
