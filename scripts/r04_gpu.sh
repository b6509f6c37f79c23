#!/bin/bash
# Round 4 GPU-box run: GPU suite, smoke, then per workload a bench line and (PROF=1) the
# rocprofv3 kernel trace + FETCH/WRITE/TCC PMC passes of the same command.
# Usage: bash scripts/r04_gpu.sh TAG "name|bench args" ...   (SKIP_TESTS=1, SKIP_SMOKE=1, PROF=1)
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    ${PYTEST_K:+-k "$PYTEST_K"} > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
  tail -2 "$OUT/pytest.log"
fi
if [ -z "${SKIP_SMOKE:-}" ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail "$OUT/smoke.log"; exit 1; }
  tail -1 "$OUT/smoke.log"
fi
for spec in "$@"; do
  name=${spec%%|*}; args=${spec#*|}
  D=$OUT/$name
  mkdir -p "$D"
  timeout -k 10 400 python3 -u bench.py $args > "$D/bench.json" 2> "$D/bench.err" || { tail -20 "$D/bench.err"; exit 1; }
  python3 -c "import json;d=json.loads(open('$D/bench.json').read().strip().splitlines()[-1]);r=d.get('roofline') or {};print('$name', d['value'], d['ms_per_step'], r.get('kernel'), r.get('avg_launch_ms'), r.get('frac'))"
  if [ -n "${PROF:-}" ]; then
    cd /tmp
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$D/trace" -o run --output-format csv -- python3 "$R/bench.py" $args --no-cpu-baseline --no-host-inclusive > "$D/prof.log" 2>&1 || { tail -20 "$D/prof.log"; exit 1; }
    timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$D/pmc_fetch" -o run --output-format csv -- python3 "$R/bench.py" $args --no-cpu-baseline --no-host-inclusive --steps 2 --warmup 1 > "$D/pmc1.log" 2>&1 || { tail -20 "$D/pmc1.log"; exit 1; }
    timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$D/pmc_write" -o run --output-format csv -- python3 "$R/bench.py" $args --no-cpu-baseline --no-host-inclusive --steps 2 --warmup 1 > "$D/pmc2.log" 2>&1 || { tail -20 "$D/pmc2.log"; exit 1; }
    timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum --kernel-trace -d "$D/pmc_tcc" -o run --output-format csv -- python3 "$R/bench.py" $args --no-cpu-baseline --no-host-inclusive --steps 2 --warmup 1 > "$D/pmc3.log" 2>&1 || { tail -20 "$D/pmc3.log"; exit 1; }
    cd "$R"
    # summarise on the box (the raw traces exceed what gpurun copies back), keep the summaries
    wl=$(echo " $args" | sed -n 's/.* --workload \([a-z0-9]*\).*/\1/p'); wl=${wl:-c3}
    kv=$(python3 -c "
import json
d = json.loads(open('$D/bench.json').read().strip().splitlines()[-1])
r = d.get('roofline') or {}
print(('%s=%d' % (r['kernel'], r['algorithmic_bytes_per_launch'])) if r.get('kernel') else '')")
    python3 scripts/pmc_summary.py "$D" "$D/$name" workload=$wl block_size=$(python3 -c "import json;print(json.loads(open('$D/bench.json').read().strip().splitlines()[-1])['config']['block_size'])") $kv > "$D/summary.log" 2>&1 || { tail -20 "$D/summary.log"; exit 1; }
    rm -rf "$D/trace" "$D/pmc_fetch" "$D/pmc_write" "$D/pmc_tcc"
  fi
done
echo "== done"
