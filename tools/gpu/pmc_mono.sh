#!/bin/bash
# Two PMC passes (stall/LDS counters, instruction mix) over one bench workload (W).
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd /tmp; export TMPDIR=/tmp
W=${W:-bloom10mono}; O=$R/gpurun_out/${O:-pmc_$W}
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS -d $O/a -o run --output-format csv -- python3 $R/bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-verify --ramp-ms 0 > $O.a.log 2>&1 &&
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES GRBM_GUI_ACTIVE -d $O/b -o run --output-format csv -- python3 $R/bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-verify --ramp-ms 0 > $O.b.log 2>&1 &&
python3 - <<PY
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob('$O/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r['Kernel_Name'].split('(')[0]][r['Counter_Name']].append(float(r['Counter_Value']))
for k, d in acc.items():
    if 'tkv::' not in k: continue
    print(k, {c: round(sum(v) / len(v)) for c, v in sorted(d.items())})
PY
