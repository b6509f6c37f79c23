#!/bin/bash
# Round 5: the file walk (K10) -- parity tests, then C4 bench lines (1 and 10 callers) with
# the kernel's phase ticks.  Usage: scripts/r05_fw.sh TAG
set -euo pipefail
tag=${1:-r05}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_file_walk.py > "$out/fw_pytest.log" 2>&1
SYDELTA_PHASE_TIMING=1 SYDELTA_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --workload c4 --steps 3 --warmup 2 \
    --no-cpu-baseline > "$out/c4c1_timing_bench.json" 2> "$out/c4c1_timing.txt"
timeout -k 10 300 python -u bench.py --workload c4 --steps 10 --warmup 3 --no-cpu-baseline > "$out/c4c1_bench.json" 2> "$out/c4c1_bench.err"
timeout -k 10 300 python -u bench.py --workload c4 --callers 10 --steps 10 --warmup 3 --no-cpu-baseline \
    > "$out/c4c10_bench.json" 2> "$out/c4c10_bench.err"
echo done
