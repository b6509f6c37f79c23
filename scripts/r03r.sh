#!/bin/bash
# Round 3: where k_scan_r's time goes (SYDELTA_ABLATE, measurement only: wrong
# results): 0 all, 8 no verification, 16 no fat lookups, 1 no drains, 3 no drains and
# no level-2 loads.
set -u
TAG=${1:-r03r}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp SYDELTA_SCAN_L1=5
cd "$R"
for ab in 0 8 16 1 3; do
  SYDELTA_ABLATE=$ab timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-inclusive \
    > "$OUT/ab$ab.json" 2> "$OUT/ab$ab.err" || { tail -20 "$OUT/ab$ab.err"; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/ab$ab.json').read().strip().splitlines()[-1]);print('ablate $ab', d['kernels']['k_scan_r']['avg_ms'])"
done
echo "== done"
