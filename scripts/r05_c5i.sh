#!/bin/bash
# Round 5: chunk walk with non-temporal op stores -- parity, then C5 lines for 1, 2, 4 parts
# (two runs each: the host side varies between runs).
set -euo pipefail
tag=${1:-r05}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_file_walk.py \
    tests/test_gpu_probe_chunk.py tests/test_gpu_multidevice.py tests/test_gpu_fullsize.py -k "chunk or c5 or walk or multi" \
    > "$out/pytest.log" 2>&1
for r in a b; do
  for k in 1 2 4; do
    SYDELTA_CHUNK_PIPE=$k SYDELTA_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --workload c5 \
        --steps 10 --warmup 3 --no-cpu-baseline > "$out/c5_k${k}_$r.json" 2> "$out/c5_k${k}_$r.err"
  done
done
echo done
