#!/bin/bash
# PMC passes (one counter group per pass, --pmc only) for a bench workload; $W = workload,
# $K = kernel-name substring
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; cd $R
W=${W:-bloom10}; K=${K:-bloom_build}
cd /tmp
for pass in "fetch:FETCH_SIZE" "write:WRITE_SIZE" "sq:SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  name=${pass%%:*}; ctrs=${pass#*:}
  timeout -k 10 300 rocprofv3 --pmc $ctrs -d $R/gpurun_out/pmc_${W}_$name -o run --output-format csv -- python3 $R/bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --ramp-ms 0 > $R/gpurun_out/pmc_${W}_$name.log 2>&1 || exit 1
done
cd $R && timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $R/gpurun_out/prof_$W -o run --output-format csv -- python3 $R/bench.py --workload $W --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --ramp-ms 0 > $R/gpurun_out/prof_$W.log 2>&1 || exit 2
