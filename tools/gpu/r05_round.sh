#!/bin/bash
# round-5 measurement on one MI355X: the GPU suite, the bench lines, kernel traces of the default
# command and of config 5 at 1B keys, and config 5's PMC passes (HBM bytes, VALU)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r05/${TAG:-round}; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
PARTS=${PARTS:-tests bench prof pmc}
has() { [[ " $PARTS " == *" $1 "* ]]; }
if has tests; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 2; }
  tail -1 $O/gpu_tests.log
fi
if has bench; then
  timeout -k 10 300 python -u bench.py > $O/bench_bloom10.log 2>&1 || exit 3
  timeout -k 10 300 python -u bench.py --workload vqf12 > $O/bench_vqf12.log 2>&1 || exit 4
  timeout -k 10 300 python -u bench.py --workload bloom10mono --no-e2e > $O/bench_bloom10mono.log 2>&1 || exit 5
  timeout -k 10 300 python -u bench.py --workload bloom10monok24 --no-e2e > $O/bench_bloom10monok24.log 2>&1 || exit 5
  timeout -k 10 400 python -u bench.py --workload bloom12hash --total-keys 1000000000 --steps 10 > $O/bench_c5_1B.log 2>&1 || exit 6
  timeout -k 10 300 python -u bench.py --workload probe10 > $O/bench_probe10.log 2>&1 || exit 7
  timeout -k 10 300 python -u bench.py --workload vqf12var --no-e2e > $O/bench_vqf12var.log 2>&1 || exit 7
  timeout -k 10 300 python -u bench.py --workload bloom12big --no-e2e > $O/bench_bloom12big.log 2>&1 || exit 7
fi
cd /tmp
if has prof; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_bloom10 -o run --output-format csv -- python3 $R/bench.py > $O/prof_bloom10.log 2>&1 || exit 8
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o run --output-format csv -- python3 $R/bench.py --workload bloom12hash --total-keys 1000000000 --steps 10 --no-cpu-baseline --no-e2e > $O/prof_c5.log 2>&1 || exit 9
fi
if has pmc; then
  ARGS="--workload bloom12hash --total-keys 1000000000 --no-cpu-baseline --no-verify --no-e2e --steps 2 --warmup 0 --ramp-ms 0"
  for pass in "fetch:FETCH_SIZE" "write:WRITE_SIZE" "sq:SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "valu:SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"; do
    name=${pass%%:*}; ctrs=${pass#*:}
    timeout -k 10 -s KILL 240 rocprofv3 --pmc $ctrs -d $O/pmc_c5_$name -o run --output-format csv -- python3 $R/bench.py $ARGS > $O/pmc_c5_$name.log 2>&1 || exit 10
  done
fi
python3 $R/tools/kstats.py $O/prof_bloom10 $O/prof_c5 2>/dev/null | head -20
for f in $O/bench_*.log; do grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$(basename $f)', d['value'], d['ms_per_step'], d.get('verified'))"; done
