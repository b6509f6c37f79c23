#!/bin/bash
# Round 5: where the chunk walk's waves spend their time (phase ticks per part), with and
# without the pre-roll; C5 repeated A/B of the pre-roll.
set -euo pipefail
tag=${1:-r05}
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
for p in 1 0; do
  SYDELTA_PREROLL=$p SYDELTA_PHASE_TIMING=1 SYDELTA_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --workload c5 \
      --steps 3 --warmup 2 --no-cpu-baseline > "$out/c5_pt$p.json" 2> "$out/c5_pt$p.err"
done
for r in a b c; do
  for p in 1 0; do
    SYDELTA_PREROLL=$p timeout -k 10 300 python -u bench.py --workload c5 --steps 30 --warmup 3 --no-cpu-baseline \
        > "$out/c5_pre${p}_$r.json" 2> "$out/c5_pre${p}_$r.err"
  done
done
echo done
