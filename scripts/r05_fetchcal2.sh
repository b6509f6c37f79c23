#!/bin/bash
# Round 5: TCC EA request counts (all / DRAM-bound / 128-byte / 32-byte) of the calibration
# kernels and of the C3, C4, C5 steps, for the calibrated traffic model.
set -uo pipefail
tag=${1:-r05}
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
cd /tmp
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 "$R/tools/micro_fetch_cal.hip" -o /tmp/micro_fetch_cal || exit 1
timeout -k 10 120 /tmp/micro_fetch_cal > "$out/counts.txt" 2>&1 || exit 1
P="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_32B_sum"
timeout -k 10 120 rocprofv3 --pmc $P --kernel-trace -d "$out/cal_ea" -o run --output-format csv -- /tmp/micro_fetch_cal \
    > "$out/cal_ea.log" 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$out/pmc_fetch" -o run --output-format csv -- /tmp/micro_fetch_cal \
    > "$out/pmc_fetch.log" 2>&1 || exit 1
for w in c3 c4 c5; do
    timeout -k 10 300 rocprofv3 --pmc $P --kernel-trace -d "$out/${w}_ea" -o run --output-format csv -- python3 "$R/bench.py" \
        --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-host-inclusive > "$out/${w}_ea.log" 2>&1 || exit 1
done
echo done
