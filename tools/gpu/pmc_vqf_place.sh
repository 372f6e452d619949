#!/bin/bash
# Two PMC passes (8 SQ counters each, --pmc only) over the vqf12 bench: stalls / LDS, then
# instruction mix.  Outputs gpurun_out/pmcplace_{stall,mix}/
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd /tmp; export TMPDIR=/tmp
W=${W:-vqf12}
B="$R/bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-verify --ramp-ms 0"
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS -d $R/gpurun_out/pmcplace_stall -o run --output-format csv -- python3 $B > $R/gpurun_out/pmcplace_stall.log 2>&1 &&
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES SQ_INSTS_VMEM -d $R/gpurun_out/pmcplace_mix -o run --output-format csv -- python3 $B > $R/gpurun_out/pmcplace_mix.log 2>&1
