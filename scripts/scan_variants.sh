#!/bin/bash
# C3 scan kernel variants (SYDELTA_SCAN_VARIANT): 0 = 4 WG/CU old verify, 1 = 3 WG/CU old, 2 = 4 WG/CU row verify, 3 = 3 WG/CU row verify
cd ${GRAFT_REPO_ROOT:-$(pwd)}
for v in ${VARIANTS:-0 1 2 3}; do
  SYDELTA_SCAN_VARIANT=$v timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-inclusive | python -c "import json,sys; d=json.load(sys.stdin); print('variant $v', d['value'], d['kernels']['k_scan_lds'], d['match_stats']['verified_hits'], d['match_stats']['weak_hits'])" || exit 1
done
