#!/bin/bash
# Round 5: C5 chunk-walk assembly threads (4 / 8 / 16), two parts, two runs each.
set -euo pipefail
tag=${1:-r05}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
for r in a b; do
  for t in 4 8 16; do
    SYDELTA_ASM_THREADS=$t SYDELTA_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --workload c5 \
        --steps 10 --warmup 3 --no-cpu-baseline > "$out/c5_t${t}_$r.json" 2> "$out/c5_t${t}_$r.err"
  done
done
echo done
