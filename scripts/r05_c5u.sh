#!/bin/bash
# Round 5: C5 default (adaptive last-part segments) -- chunk parity and three bench lines.
set -euo pipefail
tag=${1:-r05}
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_file_walk.py \
    tests/test_gpu_probe_chunk.py tests/test_gpu_async_index.py tests/test_gpu_multidevice.py > "$out/pytest.log" 2>&1
for r in a b c; do
    timeout -k 10 300 python -u bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline > "$out/c5_$r.json" 2> "$out/c5_$r.err"
done
echo done
