set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s9
timeout -k 10 400 python -m pytest tests/test_gpu_match.py -x -q -p no:cacheprovider > gpurun_out/s9/pytest.log 2>&1 || { tail -40 gpurun_out/s9/pytest.log; exit 1; }
tail -1 gpurun_out/s9/pytest.log
for a in "" "--basis-mib 128" "--basis-mib 32"; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-inclusive $a 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$a', d['value'], d['roofline']['achieved'], d['kernels'])"
done
timeout -k 10 300 python bench.py --workload c4 --files 2000 --steps 2 --warmup 1 2>&1 | grep -v amdgpu.ids | cut -c1-1500
