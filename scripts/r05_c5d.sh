#!/bin/bash
# Round 5: C5 host timing of the pipelined chunk walk, coherent vs non-coherent mapping.
set -euo pipefail
tag=${1:-r05}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
for k in 1 2; do
    SYDELTA_CHUNK_PIPE=$k SYDELTA_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --workload c5 --steps 5 --warmup 3 \
        --no-cpu-baseline > "$out/c5_k$k.json" 2> "$out/c5_k$k.err"
    SYDELTA_MAPPED_NC=1 SYDELTA_CHUNK_PIPE=$k SYDELTA_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --workload c5 \
        --steps 5 --warmup 3 --no-cpu-baseline > "$out/c5_nc_k$k.json" 2> "$out/c5_nc_k$k.err"
done
echo done
