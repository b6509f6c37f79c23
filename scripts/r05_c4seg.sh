#!/bin/bash
# Round 5: segmented file walks -- parity, then C4 per-rank shares and the 10-caller line.
set -euo pipefail
tag=${1:-r05}
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_file_walk.py \
    > "$out/pytest.log" 2>&1
for f in 10000 5000 2500 1250; do
    SYDELTA_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --workload c4 --files $f --steps 20 --warmup 3 --no-cpu-baseline \
        > "$out/c4_f$f.json" 2> "$out/c4_f$f.err"
done
SYDELTA_FILE_SEGS=1 timeout -k 10 300 python -u bench.py --workload c4 --files 1250 --steps 20 --warmup 3 --no-cpu-baseline \
    > "$out/c4_f1250_g1.json" 2> "$out/c4_f1250_g1.err"
timeout -k 10 300 python -u bench.py --workload c4 --callers 10 --steps 10 --warmup 2 --no-cpu-baseline \
    > "$out/c4_c10.json" 2> "$out/c4_c10.err"
echo done
