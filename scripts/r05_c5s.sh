#!/bin/bash
# Round 5: C5 with the HIP API trace beside the kernel trace (no counters): when the host issues each call.
set -euo pipefail
tag=${1:-r05}
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -d "$out/trace" -o run --output-format csv -- \
    python3 "$R/bench.py" --workload c5 --steps 4 --warmup 2 --no-cpu-baseline > "$out/prof.log" 2>&1
echo done
