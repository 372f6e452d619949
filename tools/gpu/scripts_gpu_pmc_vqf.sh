#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; cd $R
cd /tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_SALU -d $R/gpurun_out/pmc_vqf_a -o run --output-format csv -- python3 $R/bench.py --workload vqf12 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --ramp-ms 0 > $R/gpurun_out/pmc_vqf_a.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_INST_CYCLES_SALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc_vqf_b -o run --output-format csv -- python3 $R/bench.py --workload vqf12 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --ramp-ms 0 > $R/gpurun_out/pmc_vqf_b.log 2>&1 || exit 2
