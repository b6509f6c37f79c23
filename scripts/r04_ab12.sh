#!/bin/bash
# C3 k_scan_r ablations at the default layout (SYDELTA_ABLATE, measurement only): 0 full,
# 1 no drains, 3 no drains + no level-2 loads, 8 no hashing, 16 no lookups (so no hits).
set -u
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
for ab in 1 3 8 16; do
  SYDELTA_ABLATE=$ab timeout -k 10 200 python3 -u bench.py --workload c3 --steps 8 --warmup 2 --no-cpu-baseline --no-host-inclusive > "$OUT/ab$ab.json" 2> "$OUT/ab$ab.err" || { tail -20 "$OUT/ab$ab.err"; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/ab$ab.json').read().strip().splitlines()[-1]);print('ablate $ab', d['ms_per_step'], d['kernels']['k_scan_r'])"
done
echo "== done"
