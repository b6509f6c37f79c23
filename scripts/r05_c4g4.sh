#!/bin/bash
# Round 5: C4 with the one-round segment rule -- parity, then the per-rank shares.
set -euo pipefail
tag=${1:-r05}
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_file_walk.py > "$out/pytest.log" 2>&1
for r in a b; do
  for f in 10000 5000 2500 1250; do
    timeout -k 10 300 python -u bench.py --workload c4 --files $f --steps 20 --warmup 3 --no-cpu-baseline \
        > "$out/c4_f${f}_$r.json" 2> "$out/c4_f${f}_$r.err"
  done
done
echo done
