#!/bin/bash
# Round 5: C5 chunk-walk assembly threads (SYDELTA_WALK_THREADS) A/B, pipelined in 1 and 2 parts.
set -euo pipefail
tag=${1:-r05}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
for k in 1 2; do
  for t in 4 8 16; do
    SYDELTA_WALK_THREADS=$t SYDELTA_CHUNK_PIPE=$k SYDELTA_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --workload c5 \
        --steps 5 --warmup 3 --no-cpu-baseline > "$out/c5_k${k}_t$t.json" 2> "$out/c5_k${k}_t$t.err"
  done
done
echo done
