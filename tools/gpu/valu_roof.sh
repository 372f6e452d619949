#!/bin/bash
# VALU roof grounding: the in-kernel-clock microbenchmark, then PMC passes (one counter group
# per pass, --pmc only) of VALU activity for the default bench kernel and the window path.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/${O:-valu}; mkdir -p $O
timeout -k 10 200 ./tools/ubench_valu > $O/ubench.log 2>&1 || exit 2
cat $O/ubench.log
cd /tmp; export TMPDIR=/tmp
VALU="SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
for W in ${WS:-bloom10 vqf12}; do
  timeout -k 10 -s KILL 240 rocprofv3 --pmc $VALU -d $O/pmc_${W}_valu -o run --output-format csv -- python3 $R/bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-verify --ramp-ms 300 > $O/pmc_${W}_valu.log 2>&1 || exit 3
done
for L in ${WIN:-512 70}; do
  timeout -k 10 -s KILL 240 rocprofv3 --pmc $VALU -d $O/pmc_win${L}_valu -o run --output-format csv -- python3 $R/tools/small_batch.py --leaf-keys 200000 --bpk 12 --leaves $L --reps 5 > $O/pmc_win${L}_valu.log 2>&1 || exit 4
done
ls $O
