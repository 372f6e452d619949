#!/bin/bash
# End-of-round measurement on one MI355X (run via gpurun).  Every GPU step has its own time
# limit and the script stops at the first failure.  Outputs land in gpurun_out/round/; the
# summaries worth keeping are copied into profiles/<round>/ afterwards.
#   gpurun -- ./tools/gpu/profile_round.sh
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/${O:-round}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 2
timeout -k 10 300 python bench.py > $O/bench_bloom10.log 2>&1 || exit 3
timeout -k 10 300 python bench.py --workload vqf12 --no-e2e > $O/bench_vqf12.log 2>&1 || exit 4
timeout -k 10 300 python bench.py --workload probe10 > $O/bench_probe10.log 2>&1 || exit 5
timeout -k 10 300 python bench.py --workload probe_vqf12 > $O/bench_probe_vqf12.log 2>&1 || exit 6
timeout -k 10 300 python bench.py --workload bloom12 --no-e2e > $O/bench_bloom12.log 2>&1 || exit 7
timeout -k 10 300 python bench.py --workload bloom10k24 > $O/bench_bloom10k24.log 2>&1 || exit 8
timeout -k 10 300 python bench.py --workload bloom12 --total-keys 1000000000 --steps 10 --no-e2e > $O/bench_bloom12_1B.log 2>&1 || exit 9
timeout -k 10 300 python bench.py --workload bloom10mono > $O/bench_bloom10mono.log 2>&1 || exit 10
timeout -k 10 300 python bench.py --workload bloom10var --no-e2e > $O/bench_bloom10var.log 2>&1 || exit 10
cd /tmp
# kernel-trace stats of the exact default bench command, and of the other workloads
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $O/prof_bloom10 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-e2e > $O/prof_bloom10.log 2>&1 || exit 11
for W in vqf12 probe10 probe_vqf12 bloom10mono; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $O/prof_$W -o run --output-format csv -- python3 $R/bench.py --workload $W --no-cpu-baseline --no-e2e > $O/prof_$W.log 2>&1 || exit 12
done
# HBM traffic + VALU counters: one counter group per pass, --pmc only, no clock ramp
for W in ${PMC_WS:-bloom10 vqf12}; do
  for pass in "fetch:FETCH_SIZE" "write:WRITE_SIZE" "sq:SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
    name=${pass%%:*}; ctrs=${pass#*:}
    timeout -k 10 -s KILL 240 rocprofv3 --pmc $ctrs -d $O/pmc_${W}_$name -o run --output-format csv -- python3 $R/bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --ramp-ms 0 > $O/pmc_${W}_$name.log 2>&1 || exit 13
  done
done
