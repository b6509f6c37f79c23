#!/bin/bash
# Round 5: C4 10 callers and 1 caller, library A/B (r05g build first), alternating, two rounds; the 1250-file share.
set -euo pipefail
tag=${1:-r05}
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
for r in a b; do
  for v in r05g cur; do
    if [ $v = cur ]; then unset SYDELTA_LIB_VARIANT; else export SYDELTA_LIB_VARIANT=$v; fi
    timeout -k 10 300 python -u bench.py --workload c4 --callers 10 --steps 20 --warmup 3 --no-cpu-baseline \
        > "$out/c4_c10_${v}_$r.json" 2> "$out/c4_c10_${v}_$r.err"
    timeout -k 10 300 python -u bench.py --workload c4 --steps 20 --warmup 3 --no-cpu-baseline \
        > "$out/c4_c1_${v}_$r.json" 2> "$out/c4_c1_${v}_$r.err"
    timeout -k 10 300 python -u bench.py --workload c4 --files 1250 --steps 20 --warmup 3 --no-cpu-baseline \
        > "$out/c4_f1250_${v}_$r.json" 2> "$out/c4_f1250_${v}_$r.err"
  done
done
unset SYDELTA_LIB_VARIANT
echo done
