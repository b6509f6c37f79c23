#!/bin/bash
# Round 5: C4 per-rank shares on one GPU (10000 / N files for N = 1, 2, 4, 8): the strong-
# scaling curve the 8-GPU run would see if ranks do not interfere; plus 10 callers.
set -euo pipefail
tag=${1:-r05}
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
for f in 10000 5000 2500 1250; do
    timeout -k 10 300 python -u bench.py --workload c4 --files $f --steps 20 --warmup 3 --no-cpu-baseline \
        > "$out/c4_f$f.json" 2> "$out/c4_f$f.err"
done
timeout -k 10 300 python -u bench.py --workload c4 --callers 10 --steps 10 --warmup 2 --no-cpu-baseline \
    > "$out/c4_c10.json" 2> "$out/c4_c10.err"
SYDELTA_HOST_THREADS=2 timeout -k 10 300 python -u bench.py --workload c4 --files 1250 --steps 20 --warmup 3 \
    --no-cpu-baseline > "$out/c4_f1250_t2.json" 2> "$out/c4_f1250_t2.err"
echo done
