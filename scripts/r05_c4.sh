#!/bin/bash
# Round 5: C4 with the file walk (K10): bench lines (1 and 10 callers), host timing, and
# the rocprofv3 kernel trace of the one-caller command.  Usage: scripts/r05_c4.sh TAG
set -euo pipefail
tag=${1:-r05b}
out=gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u bench.py --workload c4 --steps 10 --warmup 3 > "$out/c4c1_bench.json" 2> "$out/c4c1_bench.err"
timeout -k 10 300 python -u bench.py --workload c4 --callers 10 --steps 10 --warmup 3 --no-cpu-baseline \
    > "$out/c4c10_bench.json" 2> "$out/c4c10_bench.err"
SYDELTA_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --workload c4 --steps 3 --warmup 2 --no-cpu-baseline \
    > "$out/c4c1_ht_bench.json" 2> "$out/c4c1_host_timing.txt"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof" -o c4c1 -- python3 bench.py --workload c4 --steps 5 \
    --warmup 2 --no-cpu-baseline > "$out/c4c1_prof_bench.json" 2> "$out/c4c1_prof.err"
echo done
