#!/bin/bash
# Round 5: the async index build + pipelined chunk walk -- the whole GPU suite, then C5 A/B
# (index built synchronously or overlapped; 1 or 2 sub-ranges) with host timing.
set -euo pipefail
tag=${1:-r05}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > "$out/pytest.log" 2>&1
for v in "1 0" "1 1" "2 0" "2 1"; do
    set -- $v
    SYDELTA_CHUNK_PIPE=$1 SYDELTA_INDEX_SYNC=$2 SYDELTA_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --workload c5 \
        --steps 10 --warmup 3 --no-cpu-baseline > "$out/c5_k$1_s$2.json" 2> "$out/c5_k$1_s$2.err"
done
echo done
