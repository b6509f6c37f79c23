#!/bin/bash
# Round 3: inline k_scan_r's drain split (SYDELTA_ABLATE, measurement only): 0 all,
# 8 no hashing, 16 no lookups, 1 no drains.
set -u
TAG=${1:-r03ak}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
for ab in 0 8 16 1; do
  SYDELTA_ABLATE=$ab timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-inclusive \
    > "$OUT/ab$ab.json" 2> "$OUT/ab$ab.err" || { tail -20 "$OUT/ab$ab.err"; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/ab$ab.json').read().strip().splitlines()[-1]);print('ablate $ab', d['kernels']['k_scan_r']['avg_ms'])"
done
echo "== done"
