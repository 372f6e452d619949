#!/bin/bash
# round 4: where the monolithic partition's time goes -- phase-knockout builds
# (tools/exp/libtkv_amq_exp{1,2,3}.so: no stores / no place / hash only) and PMC passes
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04/${TAG:-exp}
mkdir -p $O
B="python -u bench.py --workload bloom10mono --steps 20 --no-e2e --no-cpu-baseline --no-verify"
for v in 1 2 3; do
  TKV_AMQ_LIB=tools/exp/libtkv_amq_exp$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats \
      -d $O/prof_exp$v -o p --output-format csv -- $B > $O/bench_exp$v.log 2>&1 || exit 2
done
for pass in "sq:SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
            "valu:SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" \
            "write:WRITE_SIZE" "fetch:FETCH_SIZE"; do
  name=${pass%%:*}; ctrs=${pass#*:}
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $ctrs -d $O/pmc_$name -o run --output-format csv -- \
      python3 bench.py --workload bloom10mono --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-verify \
      --ramp-ms 0 > $O/pmc_$name.log 2>&1 || echo "pmc $name failed"
done
echo done
