#!/bin/bash
# Round 5: C5 chunk walk -- results copied out of mapped memory or read in place, 1 and 2 parts.
set -euo pipefail
tag=${1:-r05}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
for k in 1 2; do
  for c in 1 0; do
    SYDELTA_CHUNK_COPYREC=$c SYDELTA_CHUNK_PIPE=$k SYDELTA_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --workload c5 \
        --steps 8 --warmup 3 --no-cpu-baseline > "$out/c5_k${k}_c$c.json" 2> "$out/c5_k${k}_c$c.err"
  done
done
echo done
