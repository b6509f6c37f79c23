set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s8
timeout -k 10 300 python -m pytest tests/test_gpu_match.py -x -q -p no:cacheprovider > gpurun_out/s8/pytest.log 2>&1 || { tail -30 gpurun_out/s8/pytest.log; exit 1; }
tail -1 gpurun_out/s8/pytest.log
for a in "" "--basis-mib 128" "--basis-mib 32"; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline $a 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$a', d['value'], d['roofline']['achieved'], d['kernels'])"
done
SYDELTA_PHASE_TIMING=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --basis-mib 32 2>&1 | grep phase | head -1
