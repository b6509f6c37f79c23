#!/bin/bash
# Round 5: C5 walks on low-priority streams (two per thread) -- parity, 2 / 3 parts, priority A/B, trace.
set -euo pipefail
tag=${1:-r05}
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_file_walk.py \
    tests/test_gpu_probe_chunk.py -k "chunk or c5" > "$out/pytest.log" 2>&1
for v in "2 1" "3 1" "2 0"; do
    set -- $v
    SYDELTA_CHUNK_PIPE=$1 SYDELTA_WALK_PRIO=$2 timeout -k 10 300 python -u bench.py --workload c5 --steps 20 --warmup 3 \
        --no-cpu-baseline > "$out/c5_k$1_p$2.json" 2> "$out/c5_k$1_p$2.err"
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/trace" -o run --output-format csv -- python3 "$R/bench.py" \
    --workload c5 --steps 6 --warmup 2 --no-cpu-baseline > "$out/prof.log" 2>&1
echo done
