#!/bin/bash
# wire-format GPU checks, then the json bench at 256 MiB and at the full 4 GiB
cd ${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 300 python -u -m pytest tests/test_gpu_wire.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider 2>&1 | tail -3 || exit 1
for g in 0.25 4; do
  timeout -k 10 300 python bench.py --workload json --size-gib $g --steps 3 --warmup 1 2>/dev/null | grep '^{' | python -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['ms_per_step'], d['roofline'], d['kernels'], d['cpu_baseline'], d['match_stats'])" || exit 1
done
