#!/bin/bash
# PMC passes for the probe workloads (shuffled lookups, BASELINE config 4): memory-side
# request bytes and L2 hit/miss counts, one counter group per pass, --pmc only.
#   gpurun -- ./tools/gpu/pmc_probe.sh
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/pmcp
cd /tmp
for W in ${WS:-probe10 probe_vqf12}; do
  for pass in "fetch:FETCH_SIZE" "write:WRITE_SIZE" "tcc:TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
    name=${pass%%:*}; ctrs=${pass#*:}
    timeout -s KILL 240 rocprofv3 --pmc $ctrs -d $R/gpurun_out/pmcp/${W}_$name -o run --output-format csv -- python3 $R/bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --ramp-ms 0 > $R/gpurun_out/pmcp/${W}_$name.log 2>&1 || exit 1
  done
done
