#!/bin/bash
# PMC passes with the round's final code: config 5 at 1B keys and the 24-byte-key monolithic build
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r05/pmcfinal; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
cd /tmp
for W in c5 k24; do
  if [ $W = c5 ]; then ARGS="--workload bloom12hash --total-keys 1000000000 --no-cpu-baseline --no-verify --no-e2e --steps 2 --warmup 0 --ramp-ms 0"
  else ARGS="--workload bloom10monok24 --no-cpu-baseline --no-verify --no-e2e --steps 3 --warmup 1 --ramp-ms 0"; fi
  for pass in "fetch:FETCH_SIZE" "write:WRITE_SIZE" "sq:SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "valu:SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"; do
    name=${pass%%:*}; ctrs=${pass#*:}
    timeout -k 10 -s KILL 240 rocprofv3 --pmc $ctrs -d $O/${W}_$name -o run --output-format csv -- python3 $R/bench.py $ARGS > $O/${W}_$name.log 2>&1 || { echo "$W $name failed"; tail -20 $O/${W}_$name.log; exit 10; }
  done
done
echo done
