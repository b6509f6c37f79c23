#!/bin/bash
# Round 5: C5 part sizes (uneven, shrinking tail) with walks on two alternating streams;
# the async-contract GPU tests first.
set -euo pipefail
tag=${1:-r05}
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_async_index.py \
    tests/test_gpu_file_walk.py -k "async or chunk or index" > "$out/pytest.log" 2>&1
for v in "2 50,50" "3 45,38,17" "4 35,30,22,13" "3 40,40,20"; do
    set -- $v
    for r in a b; do
        SYDELTA_CHUNK_PIPE=$1 SYDELTA_CHUNK_PIPE_W=$2 timeout -k 10 300 python -u bench.py --workload c5 --steps 20 --warmup 3 \
            --no-cpu-baseline > "$out/c5_k$1_${2//,/-}_$r.json" 2> "$out/c5_k$1_${2//,/-}_$r.err"
    done
done
cd /tmp
SYDELTA_CHUNK_PIPE=4 SYDELTA_CHUNK_PIPE_W=35,30,22,13 timeout -k 10 300 rocprofv3 --kernel-trace -d "$out/trace" -o run \
    --output-format csv -- python3 "$R/bench.py" --workload c5 --steps 6 --warmup 2 --no-cpu-baseline > "$out/prof.log" 2>&1
echo done
