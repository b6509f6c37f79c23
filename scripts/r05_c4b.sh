#!/bin/bash
# Round 5: C4 with 10 callers (batch indexes built in the caller's stream order again), 1 caller.
set -euo pipefail
tag=${1:-r05}
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --workload c4 --callers 10 --steps 10 --warmup 2 --no-cpu-baseline \
    > "$out/c4_c10.json" 2> "$out/c4_c10.err"
timeout -k 10 300 python -u bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline > "$out/c4_c1.json" 2> "$out/c4_c1.err"
SYDELTA_INDEX_SYNC=1 timeout -k 10 300 python -u bench.py --workload c4 --callers 10 --steps 10 --warmup 2 --no-cpu-baseline \
    > "$out/c4_c10_sync.json" 2> "$out/c4_c10_sync.err"
echo done
