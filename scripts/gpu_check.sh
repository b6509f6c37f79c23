#!/bin/bash
# GPU-box check: parity tests, bench line, rocprofv3 kernel stats, PMC HBM bytes.
# Usage (from the repo root on the box): bash scripts/gpu_check.sh [tag] [bench args...]
set -u
TAG=${1:-r01}; shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
step() { local t=$1; shift; echo "== $* (limit ${t}s)" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== rc=$rc" >&2; return $rc; }
[ -n "${SKIP_TESTS:-}" ] || step 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log" 2>/dev/null
step 600 python bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" || { cat "$OUT/bench.err" | tail -20; exit 1; }
cat "$OUT/bench.json"
cd /tmp
# profiled runs: the same workload without the CPU baseline and host-inclusive legs,
# so every launch of a kernel has the bench's size and the averages agree
step 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --no-host-inclusive "$@" > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
step 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --no-host-inclusive --steps 2 --warmup 1 "$@" > "$OUT/pmc1.log" 2>&1 || { tail -20 "$OUT/pmc1.log"; exit 1; }
step 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc_write" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --no-host-inclusive --steps 2 --warmup 1 "$@" > "$OUT/pmc2.log" 2>&1 || { tail -20 "$OUT/pmc2.log"; exit 1; }
if [ -n "${TCC:-}" ]; then
    step 300 rocprofv3 --pmc TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-trace -d "$OUT/pmc_tcc" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --no-host-inclusive --steps 2 --warmup 1 "$@" > "$OUT/pmc3.log" 2>&1 || { tail -20 "$OUT/pmc3.log"; exit 1; }
fi
echo "== done"
find "$OUT" -name "*.csv" | head -20
