#!/bin/bash
# Round 5: C4 ten callers, three runs, and one caller.
set -euo pipefail
tag=${1:-r05}
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
for r in a b c; do
    timeout -k 10 300 python -u bench.py --workload c4 --callers 10 --steps 20 --warmup 3 --no-cpu-baseline \
        > "$out/c4_c10_$r.json" 2> "$out/c4_c10_$r.err"
done
timeout -k 10 300 python -u bench.py --workload c4 --steps 20 --warmup 3 --no-cpu-baseline > "$out/c4_c1.json" 2> "$out/c4_c1.err"
echo done
