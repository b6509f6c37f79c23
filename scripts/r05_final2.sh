#!/bin/bash
# Round 5 final tree (pre-roll + slim walk): the whole GPU suite, smoke(), the default bench line, --gpus 1, C5, C4.
set -uo pipefail
tag=${1:-r05}
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
step() { local t=$1; shift; echo "== $* (limit ${t}s)" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== rc=$rc" >&2; return $rc; }
step 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$out/pytest.log" 2>&1 || { tail -30 "$out/pytest.log"; exit 1; }
tail -2 "$out/pytest.log"
step 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || { tail -20 "$out/smoke.log"; exit 1; }
step 600 python -u bench.py > "$out/bench_default.json" 2> "$out/bench_default.err" || { tail -20 "$out/bench_default.err"; exit 1; }
step 300 python -u bench.py --gpus 1 --steps 5 --warmup 2 --no-cpu-baseline --no-host-inclusive > "$out/bench_gpus1.json" 2> "$out/bench_gpus1.err" || exit 1
step 300 python -u bench.py --workload c5 --steps 30 --warmup 3 --no-cpu-baseline > "$out/c5.json" 2> "$out/c5.err" || exit 1
step 300 python -u bench.py --workload c4 --steps 20 --warmup 3 --no-cpu-baseline > "$out/c4.json" 2> "$out/c4.err" || exit 1
echo "== done"
