#!/bin/bash
# Round 5: C4 10 callers across library builds (r05g, c729aaa, 7022e37, current), two rounds.
set -euo pipefail
tag=${1:-r05}
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
for r in a b; do
  for v in r05g c729aaa 7022e37 cur; do
    if [ $v = cur ]; then unset SYDELTA_LIB_VARIANT; else export SYDELTA_LIB_VARIANT=$v; fi
    timeout -k 10 300 python -u bench.py --workload c4 --callers 10 --steps 20 --warmup 3 --no-cpu-baseline \
        > "$out/c4_c10_${v}_$r.json" 2> "$out/c4_c10_${v}_$r.err"
  done
done
unset SYDELTA_LIB_VARIANT
echo done
