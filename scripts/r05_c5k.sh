#!/bin/bash
# Round 5: C5 segment size (blocks per walk wave) 128 / 64 / 32, two runs each.
set -euo pipefail
tag=${1:-r05}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_file_walk.py \
    -k chunk > "$out/pytest.log" 2>&1
SYDELTA_CHUNK_SEG=32 timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
    tests/test_gpu_file_walk.py -k chunk > "$out/pytest_seg32.log" 2>&1
for r in a b; do
  for g in 128 64 32; do
    SYDELTA_CHUNK_SEG=$g SYDELTA_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --workload c5 \
        --steps 10 --warmup 3 --no-cpu-baseline > "$out/c5_g${g}_$r.json" 2> "$out/c5_g${g}_$r.err"
  done
done
echo done
