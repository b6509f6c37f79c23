#!/bin/bash
# round-2 scan iteration on the GPU box: large-index parity, match parity, C3 bench A/B
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r2}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
step() { local t=$1; shift; echo "== $* (limit ${t}s)" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== rc=$rc" >&2; return $rc; }
step 400 python -u -m pytest tests/test_gpu_scan_large.py ${TESTS:-} -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -8 "$OUT/pytest.log"
step 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-inclusive > "$OUT/bench_l1.json" 2> "$OUT/bench_l1.err" || { tail -20 "$OUT/bench_l1.err"; exit 1; }
cat "$OUT/bench_l1.json"
SYDELTA_SCAN_L1=0 step 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-inclusive > "$OUT/bench_old.json" 2> "$OUT/bench_old.err" || { tail -20 "$OUT/bench_old.err"; exit 1; }
cat "$OUT/bench_old.json"
