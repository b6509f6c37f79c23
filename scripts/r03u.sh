#!/bin/bash
# Round 3: where k_verify_r's time goes (SYDELTA_ABLATE, measurement only: wrong
# results): 8 no hashing, 16 no fat lookups (so no hits), 32 no row loads, 56 none.
set -u
TAG=${1:-r03u}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp SYDELTA_SCAN_L1=5
cd "$R"
for ab in 0 8 16 32 40 56; do
  SYDELTA_ABLATE=$ab timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-inclusive \
    > "$OUT/ab$ab.json" 2> "$OUT/ab$ab.err" || { tail -20 "$OUT/ab$ab.err"; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/ab$ab.json').read().strip().splitlines()[-1]);k=d['kernels'];print('ablate $ab', k['k_scan_r']['avg_ms'], k['k_verify_r']['avg_ms'])"
done
echo "== done"
