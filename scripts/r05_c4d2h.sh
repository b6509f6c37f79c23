#!/bin/bash
# Round 5: C4 walk results mapped vs copied down (SYDELTA_WALK_D2H), ten callers and one, alternating.
set -euo pipefail
tag=${1:-r05}
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
for r in a b; do
  for v in 1 0; do
    SYDELTA_WALK_D2H=$v timeout -k 10 300 python -u bench.py --workload c4 --callers 10 --steps 20 --warmup 3 --no-cpu-baseline \
        > "$out/c4_c10_d${v}_$r.json" 2> "$out/c4_c10_d${v}_$r.err"
    SYDELTA_WALK_D2H=$v timeout -k 10 300 python -u bench.py --workload c4 --steps 20 --warmup 3 --no-cpu-baseline \
        > "$out/c4_c1_d${v}_$r.json" 2> "$out/c4_c1_d${v}_$r.err"
    SYDELTA_WALK_D2H=$v timeout -k 10 300 python -u bench.py --workload c4 --files 1250 --steps 20 --warmup 3 --no-cpu-baseline \
        > "$out/c4_f1250_d${v}_$r.json" 2> "$out/c4_f1250_d${v}_$r.err"
  done
done
echo done
