#!/bin/bash
# Round 5: C4 expansion threads (8 vs the pool + 1) at 10000 / 1250 files and 10 callers.
set -euo pipefail
tag=${1:-r05}
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
for r in a b; do
  for t in 8 17; do
    for f in 10000 1250; do
      SYDELTA_ASM_THREADS=$t timeout -k 10 300 python -u bench.py --workload c4 --files $f --steps 20 --warmup 3 \
          --no-cpu-baseline > "$out/c4_f${f}_t${t}_$r.json" 2> "$out/c4_f${f}_t${t}_$r.err"
    done
    SYDELTA_ASM_THREADS=$t timeout -k 10 300 python -u bench.py --workload c4 --callers 10 --steps 20 --warmup 3 \
        --no-cpu-baseline > "$out/c4_c10_t${t}_$r.json" 2> "$out/c4_c10_t${t}_$r.err"
  done
done
echo done
