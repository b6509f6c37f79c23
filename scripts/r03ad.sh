#!/bin/bash
# Round 3: index memory recycled per device (sydelta_api.cpp, index_release): the whole
# GPU suite, the C3 step's host pieces, the default bench line.
set -u
TAG=${1:-r03ad}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
step() { local t=$1; shift; echo "== $* (limit ${t}s)" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== rc=$rc" >&2; return $rc; }
step 1100 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
SYDELTA_HOST_TIMING=1 step 200 python3 scripts/r03_step_host.py > "$OUT/step_host.log" 2>&1 || { tail -20 "$OUT/step_host.log"; exit 1; }
grep rep "$OUT/step_host.log"
step 400 python3 -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['roofline']['traffic'], d['roofline'].get('match'))"
echo "== done"
