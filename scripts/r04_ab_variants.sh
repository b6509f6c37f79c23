#!/bin/bash
# C3 A/B of compile-time variants (sy_amd/variants/, SYDELTA_LIB_VARIANT) on one box, interleaved.
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
for rep in 1 2; do
  for v in main "$@"; do
    if [ "$v" = main ]; then unset SYDELTA_LIB_VARIANT; else export SYDELTA_LIB_VARIANT=$v; fi
    timeout -k 10 200 python3 -u bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline --no-host-inclusive > "$OUT/${v}_$rep.json" 2> "$OUT/${v}_$rep.err" || { tail -20 "$OUT/${v}_$rep.err"; exit 1; }
    python3 -c "import json;d=json.loads(open('$OUT/${v}_$rep.json').read().strip().splitlines()[-1]);print('$v', $rep, d['ms_per_step'], d['kernels']['k_scan_r'], d['match_stats']['weak_hits'])"
  done
done
unset SYDELTA_LIB_VARIANT
echo "== done"
