#!/bin/bash
# Round 3: the path API with chunks read in parallel pieces -- its GPU tests, then the
# 4 GiB path leg with 8 readers (default) and with 1 (the previous behaviour).
set -u
TAG=${1:-r03n}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
step() { local t=$1; shift; echo "== $* (limit ${t}s)" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== rc=$rc" >&2; return $rc; }
step 600 python3 -u -m pytest tests/test_gpu_stream_path.py tests/test_gpu_reentrant.py -x -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for r in 8 1 16; do
  SYDELTA_READ_THREADS=$r step 400 python3 -u bench.py --workload path --size-gib 4 --steps 3 --warmup 1 \
    > "$OUT/bench_path_r$r.json" 2> "$OUT/bench_path_r$r.err" || { tail -20 "$OUT/bench_path_r$r.err"; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/bench_path_r$r.json').read().strip().splitlines()[-1]);print('readers $r', d['value'], d['ms_per_step'])"
done
echo "== done"
