#!/bin/bash
# Round 3: k_scan_r + k_verify_r as the default large-index scan: the whole GPU suite,
# smoke(), the default bench line, then the rocprof kernel trace and the FETCH/WRITE and
# TCC PMC passes of the C3 command (profiles/r03y_*).
set -u
TAG=${1:-r03y}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
step() { local t=$1; shift; echo "== $* (limit ${t}s)" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== rc=$rc" >&2; return $rc; }
step 1100 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
step 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
step 400 python3 -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['roofline'])"
cd /tmp
step 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$R/bench.py" \
  --no-cpu-baseline --no-host-inclusive > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
step 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 "$R/bench.py" \
  --no-cpu-baseline --no-host-inclusive --steps 2 --warmup 1 > "$OUT/pmc1.log" 2>&1 || { tail -20 "$OUT/pmc1.log"; exit 1; }
step 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc_write" -o run --output-format csv -- python3 "$R/bench.py" \
  --no-cpu-baseline --no-host-inclusive --steps 2 --warmup 1 > "$OUT/pmc2.log" 2>&1 || { tail -20 "$OUT/pmc2.log"; exit 1; }
step 120 rocprofv3 --pmc TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-trace -d "$OUT/pmc_tcc" -o run --output-format csv -- python3 "$R/bench.py" \
  --no-cpu-baseline --no-host-inclusive --steps 2 --warmup 1 > "$OUT/pmc3.log" 2>&1 || { tail -20 "$OUT/pmc3.log"; exit 1; }
echo "== done"
