#!/bin/bash
# Round 5: the slim walk of a pre-rolled part: parity, pre-roll x slim A/B, phase ticks, C4, trace.
set -euo pipefail
tag=${1:-r05}
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_file_walk.py \
    tests/test_gpu_probe_chunk.py tests/test_gpu_async_index.py > "$out/pytest.log" 2>&1
SYDELTA_PHASE_TIMING=1 SYDELTA_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --workload c5 \
    --steps 3 --warmup 2 --no-cpu-baseline > "$out/c5_pt.json" 2> "$out/c5_pt.err"
for r in a b; do
  for p in 1 0; do for sl in 1 0; do
    SYDELTA_SLIM_WALK=$sl SYDELTA_PREROLL=$p timeout -k 10 300 python -u bench.py --workload c5 --steps 30 --warmup 3 --no-cpu-baseline \
        > "$out/c5_pre${p}_sl${sl}_$r.json" 2> "$out/c5_pre${p}_sl${sl}_$r.err"
  done; done
done
timeout -k 10 300 python -u bench.py --workload c4 --steps 20 --warmup 3 --no-cpu-baseline > "$out/c4.json" 2> "$out/c4.err"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof" -o c5 --output-format csv -- python3 -u "$R/bench.py" \
    --workload c5 --steps 5 --warmup 2 --no-cpu-baseline > "$out/c5_prof.json" 2> "$out/c5_prof.err"
echo done
