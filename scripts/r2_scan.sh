#!/bin/bash
# round-2 scan iteration on the GPU box: large-index parity, C3 bench A/B, phase timing
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r2}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
step() { local t=$1; shift; echo "== $* (limit ${t}s)" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== rc=$rc" >&2; return $rc; }
if [ -z "${NOTEST:-}" ]; then
step 400 python -u -m pytest ${TESTS:-tests/test_gpu_scan_large.py} -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -4 "$OUT/pytest.log"
fi
SYDELTA_PHASE_TIMING=1 step 200 python bench.py --size-gib 1 --steps 2 --warmup 1 --no-cpu-baseline --no-host-inclusive > "$OUT/timing.json" 2> "$OUT/timing.err" || { tail -20 "$OUT/timing.err"; exit 1; }
grep "phase cycles" "$OUT/timing.err" | tail -2
step 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-inclusive > "$OUT/bench_l1.json" 2> "$OUT/bench_l1.err" || { tail -20 "$OUT/bench_l1.err"; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_l1.json'));print('L1', d['value'], d['ms_per_step'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"
