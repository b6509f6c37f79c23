#!/bin/bash
# Round 5: units assembled as they finish (done marks) -- chunk parity, then C5 lines.
set -euo pipefail
tag=${1:-r05}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_file_walk.py \
    tests/test_gpu_probe_chunk.py tests/test_gpu_multidevice.py tests/test_gpu_fullsize.py -k "chunk or c5 or walk or multi" \
    > "$out/pytest.log" 2>&1
for v in "1 0" "2 0" "1 1"; do
    set -- $v
    SYDELTA_CHUNK_PIPE=$1 SYDELTA_INDEX_SYNC=$2 SYDELTA_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --workload c5 \
        --steps 10 --warmup 3 --no-cpu-baseline > "$out/c5_k$1_s$2.json" 2> "$out/c5_k$1_s$2.err"
done
timeout -k 10 300 python -u bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline > "$out/c5_default.json" 2> "$out/c5_default.err"
echo done
