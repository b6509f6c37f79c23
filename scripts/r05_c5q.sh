#!/bin/bash
# Round 5: C5 last-part segment size (128 / 64 / 32) at weights 70,30 and 60,40.
set -euo pipefail
tag=${1:-r05}
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
SYDELTA_CHUNK_SEG_LAST=32 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_file_walk.py tests/test_gpu_async_index.py -k "chunk or index" > "$out/pytest.log" 2>&1
for w in 70,30 60,40; do
  for g in 128 64 32; do
    for r in a b; do
      SYDELTA_CHUNK_PIPE_W=$w SYDELTA_CHUNK_SEG_LAST=$g timeout -k 10 300 python -u bench.py --workload c5 --steps 20 \
          --warmup 3 --no-cpu-baseline > "$out/c5_w${w/,/-}_g${g}_$r.json" 2> "$out/c5_w${w/,/-}_g${g}_$r.err"
    done
  done
done
echo done
