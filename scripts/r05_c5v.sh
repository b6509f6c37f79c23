#!/bin/bash
# Round 5: C5 part weights with adaptive last-part segments.
set -euo pipefail
tag=${1:-r05}
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
for r in a b; do
  for w in 65,35 70,30 75,25 80,20; do
    SYDELTA_CHUNK_PIPE_W=$w timeout -k 10 300 python -u bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline \
        > "$out/c5_w${w/,/-}_$r.json" 2> "$out/c5_w${w/,/-}_$r.err"
  done
done
echo done
