#!/bin/bash
# Round 5: C5 with the step on its own stream (async signature): step timeline, bench lines,
# and C3 / C4 bench lines on the same tree.
set -euo pipefail
tag=${1:-r05}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/c5_step_timing.py --steps 10 > "$out/c5_step_timing.txt" 2>&1
C5_NULL_STREAM=1 timeout -k 10 300 python -u tools/c5_step_timing.py --steps 10 > "$out/c5_step_timing_null.txt" 2>&1
for r in a b; do
  timeout -k 10 300 python -u bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline > "$out/c5_$r.json" 2> "$out/c5_$r.err"
done
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-inclusive > "$out/c3.json" 2> "$out/c3.err"
timeout -k 10 300 python -u bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline > "$out/c4.json" 2> "$out/c4.err"
echo done
