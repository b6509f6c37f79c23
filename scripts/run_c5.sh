#!/bin/bash
# C5 bench legs on one GPU (quick check + full 8 GiB chunk), plus the default C3 line.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/c5
timeout -k 10 300 python bench.py --workload c5 --size-gib 1 --steps 3 --warmup 1 > gpurun_out/c5/c5_1g.json 2> gpurun_out/c5/c5_1g.err || { tail -20 gpurun_out/c5/c5_1g.err; exit 1; }
cat gpurun_out/c5/c5_1g.json
SYDELTA_PROBE=0 timeout -k 10 300 python bench.py --workload c5 --size-gib 1 --steps 2 --warmup 1 > gpurun_out/c5/c5_1g_noprobe.json 2> gpurun_out/c5/c5_1g_noprobe.err || { tail -20 gpurun_out/c5/c5_1g_noprobe.err; exit 1; }
cat gpurun_out/c5/c5_1g_noprobe.json
timeout -k 10 300 python bench.py --workload c5 --steps 5 --warmup 2 > gpurun_out/c5/c5_8g.json 2> gpurun_out/c5/c5_8g.err || { tail -20 gpurun_out/c5/c5_8g.err; exit 1; }
cat gpurun_out/c5/c5_8g.json
