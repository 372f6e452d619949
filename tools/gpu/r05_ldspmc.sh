#!/bin/bash
# LDS counters of the monolithic build's kernels (bloom10mono): is the tile kernel LDS-bound?
set -o pipefail
O=gpurun_out/r05/ldspmc; mkdir -p $O
export TMPDIR=/tmp
ARGS="bench.py --workload bloom10mono --steps 5 --warmup 1 --ramp-ms 0 --no-cpu-baseline --no-e2e"
timeout -k 10 -s KILL 180 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES GRBM_GUI_ACTIVE -d $O/lds -o run --output-format csv -- python3 $ARGS > $O/lds.log 2>&1 \
  && timeout -k 10 -s KILL 180 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $ARGS > $O/trace.log 2>&1
echo "rc=$?"
