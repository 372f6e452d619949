#!/bin/bash
# End-of-round measurement on one MI355X (run via gpurun).  Every GPU step has its own time
# limit and the script stops at the first failure.  Outputs land in gpurun_out/$O; the
# summaries worth keeping are copied into profiles/<round>/ afterwards.
#   gpurun -- 'O=r02_round PARTS="tests bench prof pmc sweep" ./tools/gpu/profile_round.sh'
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/${O:-round}
mkdir -p $O
export TMPDIR=/tmp
PARTS=${PARTS:-tests bench prof pmc sweep}
has() { [[ " $PARTS " == *" $1 "* ]]; }
if has tests; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 2
fi
if has bench; then
  timeout -k 10 300 python bench.py > $O/bench_bloom10.log 2>&1 || exit 3
  timeout -k 10 300 python bench.py --workload vqf12 --no-e2e > $O/bench_vqf12.log 2>&1 || exit 4
  timeout -k 10 300 python bench.py --workload probe10 > $O/bench_probe10.log 2>&1 || exit 5
  timeout -k 10 300 python bench.py --workload probe_vqf12 > $O/bench_probe_vqf12.log 2>&1 || exit 6
  timeout -k 10 300 python bench.py --workload bloom12 --no-e2e > $O/bench_bloom12.log 2>&1 || exit 7
  timeout -k 10 300 python bench.py --workload bloom10k24 > $O/bench_bloom10k24.log 2>&1 || exit 8
  timeout -k 10 300 python bench.py --workload vqf12k24 > $O/bench_vqf12k24.log 2>&1 || exit 8
  timeout -k 10 300 python bench.py --workload bloom12 --total-keys 1000000000 --steps 10 --no-e2e > $O/bench_bloom12_1B.log 2>&1 || exit 9
  timeout -k 10 300 python bench.py --workload bloom10mono > $O/bench_bloom10mono.log 2>&1 || exit 10
  timeout -k 10 300 python bench.py --workload bloom10monok24 > $O/bench_bloom10monok24.log 2>&1 || exit 10
  timeout -k 10 300 python bench.py --workload bloom10var --no-e2e > $O/bench_bloom10var.log 2>&1 || exit 10
  timeout -k 10 300 python bench.py --workload bloom12hash > $O/bench_bloom12hash.log 2>&1 || exit 10
  timeout -k 10 300 python bench.py --workload vqf12var --no-e2e > $O/bench_vqf12var.log 2>&1 || exit 10
  timeout -k 10 300 python bench.py --workload bloom12big --no-e2e > $O/bench_bloom12big.log 2>&1 || exit 10
fi
if has sweep; then
  # batch-size curve (first 64 / 256 / 1024 leaves of the same keys), and the per-leaf call sizes
  for W in bloom10 vqf12; do
    timeout -k 10 300 python bench.py --workload $W --sweep --no-e2e --no-cpu-baseline > $O/sweep_$W.log 2>&1 || exit 14
  done
  timeout -k 10 300 python tools/small_batch.py --kind 0 > $O/small_bloom10.log 2>&1 || exit 15
  timeout -k 10 300 python tools/small_batch.py --kind 1 > $O/small_vqf12.log 2>&1 || exit 15
fi
cd /tmp
if has prof; then
  # kernel-trace stats of the exact default bench command, and of the other workloads
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_bloom10 -o run --output-format csv -- python3 $R/bench.py > $O/prof_bloom10.log 2>&1 || exit 11
  for W in vqf12 probe10 probe_vqf12 bloom10mono bloom10monok24 bloom12hash vqf12var bloom10var bloom12big; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$W -o run --output-format csv -- python3 $R/bench.py --workload $W --no-cpu-baseline --no-e2e > $O/prof_$W.log 2>&1 || exit 12
  done
fi
if has pmc; then
  # HBM traffic + VALU counters: one counter group per pass, --pmc only, no clock ramp
  for W in ${PMC_WS:-bloom10 vqf12 bloom10mono bloom10monok24 bloom10k24 vqf12k24 bloom10var vqf12var bloom12big}; do
    for pass in "fetch:FETCH_SIZE" "write:WRITE_SIZE" "sq:SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "valu:SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"; do
      name=${pass%%:*}; ctrs=${pass#*:}
      timeout -k 10 -s KILL 240 rocprofv3 --pmc $ctrs -d $O/pmc_${W}_$name -o run --output-format csv -- python3 $R/bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-verify --ramp-ms 0 > $O/pmc_${W}_$name.log 2>&1 || exit 13
    done
  done
  for W in ${PMC_PROBES:-probe10 probe_vqf12}; do
    for pass in "fetch:FETCH_SIZE" "write:WRITE_SIZE" "tcc:TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
      name=${pass%%:*}; ctrs=${pass#*:}
      timeout -k 10 -s KILL 240 rocprofv3 --pmc $ctrs -d $O/pmc_${W}_$name -o run --output-format csv -- python3 $R/bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-verify --ramp-ms 0 > $O/pmc_${W}_$name.log 2>&1 || exit 13
    done
  done
fi
