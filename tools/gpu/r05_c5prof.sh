#!/bin/bash
# config 5 at 1B keys on one GPU: kernel trace + PMC passes (HBM bytes, VALU)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r05/${TAG:-c5prof}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
ARGS="--workload bloom12hash --total-keys 1000000000 --no-cpu-baseline --no-verify --no-e2e"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py $ARGS --steps 5 > $O/prof.log 2>&1 || exit 2
if [ -z "$NOPMC" ]; then
for pass in "fetch:FETCH_SIZE" "write:WRITE_SIZE" "sq:SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "valu:SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"; do
  name=${pass%%:*}; ctrs=${pass#*:}
  timeout -k 10 -s KILL 240 rocprofv3 --pmc $ctrs -d $O/pmc_$name -o run --output-format csv -- python3 $R/bench.py $ARGS --steps 2 --warmup 0 --ramp-ms 0 > $O/pmc_$name.log 2>&1 || exit 3
done
fi
python3 $R/tools/kstats.py $O/prof
