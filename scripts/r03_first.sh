#!/bin/bash
# Round 3, first hardware call: every GPU test (zstd included), the C3 line, its rocprof
# kernel trace and the PMC passes of the C3 command (FETCH_SIZE, WRITE_SIZE, TCC
# requests/hits/misses, TCP->TCC read requests), each step under its own limit; stops at
# the first failure.  SCAN_KERNEL names the scan kernel of the PMC summary (k_scan_l2,
# the default scanner since r03j; r03a profiled k_scan_l1); P2=1 adds the two-partition leg.
# Usage (from the repo root on the box): bash scripts/r03_first.sh [tag]
set -u
TAG=${1:-r03a}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
step() { local t=$1; shift; echo "== $* (limit ${t}s)" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== rc=$rc" >&2; return $rc; }
[ -n "${SKIP_TESTS:-}" ] || { step 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
  -p no:cacheprovider > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }; tail -3 "$OUT/pytest.log"; }
step 400 python -u bench.py > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err" || { tail -20 "$OUT/bench_c3.err"; exit 1; }
tail -c 1500 "$OUT/bench_c3.json"; echo
cd /tmp
B="$R/bench.py --no-cpu-baseline --no-host-inclusive"
step 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 $B \
  > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
pmc() { local name=$1; shift; echo "== pmc $name: $*" >&2
  timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-trace -d "$OUT/pmc_$name" -o run --output-format csv -- python3 $B \
    --steps 2 --warmup 1 > "$OUT/pmc_$name.log" 2>&1; local rc=$?; echo "== rc=$rc" >&2
  [ $rc -eq 0 ] || tail -20 "$OUT/pmc_$name.log"; return $rc; }
pmc fetch FETCH_SIZE || exit 1
pmc write WRITE_SIZE || exit 1
pmc tcc TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum || exit 1
pmc tcp TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum || exit 1
cd "$R"
python3 scripts/pmc_summary.py "$OUT" "$OUT/c3" ${SCAN_KERNEL:-k_scan_l2}=4294967296 k_sig_fast=4294967296 > "$OUT/pmc_summary.txt" 2>&1; cat "$OUT/pmc_summary.txt"
[ -z "${P2:-}" ] || step 300 env SYDELTA_SCAN_L1=2 python3 bench.py --no-cpu-baseline --no-host-inclusive --steps 10 --warmup 3 \
  > "$OUT/bench_c3_p2.json" 2> "$OUT/bench_c3_p2.err" || { tail -20 "$OUT/bench_c3_p2.err"; exit 1; }
[ -z "${P2:-}" ] || { tail -c 1500 "$OUT/bench_c3_p2.json"; echo; }
echo "== done"
