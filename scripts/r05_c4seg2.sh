#!/bin/bash
# Round 5: C4 segments per file A/B at 10000 / 2500 / 1250 files.
set -euo pipefail
tag=${1:-r05}
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
for v in "10000 1" "10000 2" "10000 4" "2500 2" "2500 4" "2500 8" "1250 4" "1250 8"; do
    set -- $v
    SYDELTA_FILE_SEGS=$2 timeout -k 10 300 python -u bench.py --workload c4 --files $1 --steps 20 --warmup 3 --no-cpu-baseline \
        > "$out/c4_f$1_g$2.json" 2> "$out/c4_f$1_g$2.err"
done
echo done
