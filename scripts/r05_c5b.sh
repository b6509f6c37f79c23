#!/bin/bash
# Round 5: C5 bench lines (device chunk walk, classifier path) with host and phase timing.
set -euo pipefail
tag=${1:-r05}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_file_walk.py \
    > "$out/fw_pytest.log" 2>&1
timeout -k 10 300 python -u bench.py --workload c5 --steps 10 --warmup 3 --no-cpu-baseline > "$out/c5_bench.json" 2> "$out/c5_bench.err"
SYDELTA_PHASE_TIMING=1 SYDELTA_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --workload c5 --steps 3 --warmup 2 \
    --no-cpu-baseline > "$out/c5_ht_bench.json" 2> "$out/c5_host_timing.txt"
echo done
