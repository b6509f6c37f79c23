#!/bin/bash
# First hardware run of the kernels written while round 2's GPU access was closed: their
# GPU tests (marker firstrun: device walk, signature and Delta JSON parse/write, zstd), then their bench legs
# (sigjson, dparse, zstd, c5 with the device walk), each step under its own limit; stops at the
# first failure so that a fault ends the call.
# Usage (from the repo root on the box): bash scripts/firstrun.sh [tag]
set -u
TAG=${1:-firstrun}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
step() { local t=$1; shift; echo "== $* (limit ${t}s)" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== rc=$rc" >&2; return $rc; }
step 900 python -u -m pytest tests -m "gpu and firstrun" -x -v --timeout 240 --timeout-method thread \
  -p no:cacheprovider > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -4 "$OUT/pytest.log"
for w in sigjson dparse zstd; do
  step 400 python -u bench.py --workload "$w" > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err" || { tail -20 "$OUT/bench_$w.err"; exit 1; }
  tail -c 600 "$OUT/bench_$w.json"; echo
done
step 400 python -u bench.py --workload c5 --device-walk > "$OUT/bench_c5_dev.json" 2> "$OUT/bench_c5_dev.err" || { tail -20 "$OUT/bench_c5_dev.err"; exit 1; }
tail -c 600 "$OUT/bench_c5_dev.json"; echo
echo "== done"
