#!/bin/bash
# Round 5: the pre-roll of a chunk's aligned misses (k_preroll): parity, then C5 with and without.
set -euo pipefail
tag=${1:-r05}
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_file_walk.py \
    tests/test_gpu_probe_chunk.py tests/test_gpu_async_index.py > "$out/pytest.log" 2>&1
for r in a b; do
  for p in 1 0 2; do
    SYDELTA_PREROLL=$p timeout -k 10 300 python -u bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline \
        > "$out/c5_pre${p}_$r.json" 2> "$out/c5_pre${p}_$r.err"
  done
done
SYDELTA_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --workload c5 --steps 3 --warmup 2 --no-cpu-baseline \
    > "$out/c5_ht.json" 2> "$out/c5_ht.err"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof" -o c5 --output-format csv -- python3 -u "$R/bench.py" \
    --workload c5 --steps 5 --warmup 2 --no-cpu-baseline > "$out/c5_prof.json" 2> "$out/c5_prof.err"
echo done
