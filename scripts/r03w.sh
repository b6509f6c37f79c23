#!/bin/bash
# Round 3: k_scan_r + k_lookup_r + k_verify_r: large-index parity (scanner r), the C3
# bench leg (mode 5 vs k_scan_l2), and k_verify_r's ablations (8 no hashing, 16 no
# lookups, 32 no row loads).
set -u
TAG=${1:-r03w}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
SYDELTA_TEST_SCANNERS=r timeout -k 10 400 python3 -u -m pytest tests/test_gpu_scan_large.py -x -v \
  --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for m in 5 4; do
  SYDELTA_SCAN_L1=$m timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-inclusive \
    > "$OUT/mode$m.json" 2> "$OUT/mode$m.err" || { tail -20 "$OUT/mode$m.err"; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/mode$m.json').read().strip().splitlines()[-1]);print('mode $m', d['value'], d['ms_per_step'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"
done
for ab in 8 16 32; do
  SYDELTA_SCAN_L1=5 SYDELTA_ABLATE=$ab timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline \
    --no-host-inclusive > "$OUT/ab$ab.json" 2> "$OUT/ab$ab.err" || { tail -20 "$OUT/ab$ab.err"; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/ab$ab.json').read().strip().splitlines()[-1]);k=d['kernels'];print('ablate $ab', {x:k[x]['avg_ms'] for x in ('k_scan_r','k_lookup_r','k_verify_r')})"
done
echo "== done"
