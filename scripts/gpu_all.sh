#!/bin/bash
# Full GPU check: parity tests, then C3 (default), C2 and C5 bench lines.
# Usage: bash scripts/gpu_all.sh <tag>
set -u
TAG=${1:-run}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for w in c3 c2 c5; do
  timeout -k 10 400 python bench.py --workload $w > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { tail -20 $OUT/bench_$w.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$w.json')); print('$w', d['value'], d['unit'], d['ms_per_step'], 'ms/step', d['roofline']['kernel'], d['roofline']['frac'], {k: v['avg_ms'] for k, v in d['kernels'].items()})"
done
