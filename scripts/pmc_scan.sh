#!/bin/bash
# C3 scan kernel: phase cycles + SQ/TCC counters (one C3 step at 2 GiB to keep it short).
cd ${GRAFT_REPO_ROOT:-$(pwd)}
R=$(pwd)
mkdir -p gpurun_out/pmc_scan
SYDELTA_PHASE_TIMING=1 timeout -k 10 120 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-host-inclusive --size-gib 2 2>&1 | grep -E "phase" | tail -1
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS --kernel-trace -d $R/gpurun_out/pmc_scan/sq -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-host-inclusive --size-gib 2 > $R/gpurun_out/pmc_scan/log 2>&1 || { tail $R/gpurun_out/pmc_scan/log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_SALU GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH --kernel-trace -d $R/gpurun_out/pmc_scan/sq2 -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-host-inclusive --size-gib 2 >> $R/gpurun_out/pmc_scan/log 2>&1 || { tail $R/gpurun_out/pmc_scan/log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum --kernel-trace -d $R/gpurun_out/pmc_scan/tcc -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-host-inclusive --size-gib 2 >> $R/gpurun_out/pmc_scan/log 2>&1 || { tail $R/gpurun_out/pmc_scan/log; exit 1; }
cd $R
python3 - <<'PY'
import csv, collections, glob
for f in sorted(glob.glob('gpurun_out/pmc_scan/*/run_counter_collection.csv')):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if 'k_scan' in r['Kernel_Name']:
            agg[r['Counter_Name']].append(float(r['Counter_Value']))
    for k, v in agg.items():
        print(f.split('/')[-2], k, sum(v) / len(v))
PY
