#!/bin/bash
# Round 5: C5 last-part segment size 64 / 80 / 96 / 128.
set -euo pipefail
tag=${1:-r05}
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
SYDELTA_CHUNK_SEG_LAST=80 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_file_walk.py -k chunk > "$out/pytest.log" 2>&1
for r in a b; do
  for g in 64 80 96 128; do
    SYDELTA_CHUNK_SEG_LAST=$g timeout -k 10 300 python -u bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline \
        > "$out/c5_g${g}_$r.json" 2> "$out/c5_g${g}_$r.err"
  done
done
echo done
