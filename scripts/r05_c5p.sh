#!/bin/bash
# Round 5: C5 two parts, uneven weights, second walk on the aux stream; trace of 70/30.
set -euo pipefail
tag=${1:-r05}
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_file_walk.py \
    tests/test_gpu_async_index.py -k "chunk or index" > "$out/pytest.log" 2>&1
for w in 50,50 60,40 70,30 75,25; do
  for r in a b; do
    SYDELTA_CHUNK_PIPE_W=$w timeout -k 10 300 python -u bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline \
        > "$out/c5_w${w/,/-}_$r.json" 2> "$out/c5_w${w/,/-}_$r.err"
  done
done
cd /tmp
SYDELTA_CHUNK_PIPE_W=70,30 timeout -k 10 300 rocprofv3 --kernel-trace -d "$out/trace" -o run --output-format csv -- \
    python3 "$R/bench.py" --workload c5 --steps 6 --warmup 2 --no-cpu-baseline > "$out/prof.log" 2>&1
echo done
