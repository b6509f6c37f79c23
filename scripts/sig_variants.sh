#!/bin/bash
# C2 signature kernel variants (SYDELTA_SIG_VARIANT): 0 = group 4 nt, 1 = group 1 plain, 2 = group 4 plain, 3 = group 2 nt, 4 = group 8 nt
cd ${GRAFT_REPO_ROOT:-$(pwd)}
for v in 0 3; do
  SYDELTA_SIG_VARIANT=$v timeout -k 10 120 python bench.py --workload c2 --steps 20 --warmup 3 | python -c "import json,sys; d=json.load(sys.stdin); print('variant $v', d['kernels'], d['value'])" || exit 1
done
