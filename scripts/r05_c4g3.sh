#!/bin/bash
# Round 5: C4 segments per file at one wave round (units <= 4096): 1250 files G=3 vs 4 vs 6, 2500 files G=1 vs 2.
set -euo pipefail
tag=${1:-r05}
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
for r in a b; do
  for v in "1250 3" "1250 4" "1250 6" "2500 1" "2500 2" "5000 1"; do
    set -- $v
    SYDELTA_FILE_SEGS=$2 timeout -k 10 300 python -u bench.py --workload c4 --files $1 --steps 20 --warmup 3 --no-cpu-baseline \
        > "$out/c4_f$1_g$2_$r.json" 2> "$out/c4_f$1_g$2_$r.err"
  done
done
echo done
