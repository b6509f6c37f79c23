#!/bin/bash
# Round 5: the pipelined chunk walk -- parity (file walk + chunk tests), C5 bench lines for
# 1, 2 and 4 sub-ranges, host timing.
set -euo pipefail
tag=${1:-r05}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_file_walk.py \
    tests/test_gpu_probe_chunk.py > "$out/pytest.log" 2>&1
for k in 4 2 1; do
    SYDELTA_CHUNK_PIPE=$k timeout -k 10 300 python -u bench.py --workload c5 --steps 10 --warmup 3 --no-cpu-baseline \
        > "$out/c5_k$k.json" 2> "$out/c5_k$k.err"
done
SYDELTA_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --workload c5 --steps 3 --warmup 2 \
    --no-cpu-baseline > "$out/c5_ht_bench.json" 2> "$out/c5_host_timing.txt"
echo done
