#!/bin/bash
# Round 5: the GPU suite, then C5 and C4 bench lines with host timing.  Usage: scripts/r05_c5.sh TAG
set -euo pipefail
tag=${1:-r05}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > "$out/gpu_pytest.log" 2>&1
tail -3 "$out/gpu_pytest.log"
timeout -k 10 300 python -u bench.py --workload c5 --steps 10 --warmup 3 --no-cpu-baseline > "$out/c5_bench.json" 2> "$out/c5_bench.err"
SYDELTA_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --workload c5 --steps 3 --warmup 2 --no-cpu-baseline \
    > "$out/c5_ht_bench.json" 2> "$out/c5_host_timing.txt"
SYDELTA_CHUNK_WALK=0 timeout -k 10 300 python -u bench.py --workload c5 --steps 10 --warmup 3 --no-cpu-baseline \
    > "$out/c5_classifier_bench.json" 2> "$out/c5_classifier_bench.err"
echo done
