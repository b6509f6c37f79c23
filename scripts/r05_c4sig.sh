#!/bin/bash
# Round 5: batched signature without a host wait -- parity, C4 step timeline, C4 shares, 10 callers.
set -euo pipefail
tag=${1:-r05}
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_file_walk.py \
    tests/test_gpu_signature.py tests/test_gpu_match.py tests/test_gpu_reentrant.py > "$out/pytest.log" 2>&1
timeout -k 10 300 python -u tools/c4_step_timing.py --files 1250 > "$out/c4_1250_timing.txt" 2>&1
for f in 10000 2500 1250; do
    timeout -k 10 300 python -u bench.py --workload c4 --files $f --steps 20 --warmup 3 --no-cpu-baseline \
        > "$out/c4_f$f.json" 2> "$out/c4_f$f.err"
done
timeout -k 10 300 python -u bench.py --workload c4 --callers 10 --steps 20 --warmup 3 --no-cpu-baseline \
    > "$out/c4_c10.json" 2> "$out/c4_c10.err"
echo done
