#!/bin/bash
# One PMC pass of stall / LDS counters (8 SQ counters, --pmc only) over a bench workload.
#   W=vqf12 ./tools/gpu/pmc_stalls.sh
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd /tmp; export TMPDIR=/tmp
W=${W:-vqf12}
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS -d $R/gpurun_out/stall_$W -o run --output-format csv -- python3 $R/bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --ramp-ms 0 > $R/gpurun_out/stall_$W.log 2>&1
