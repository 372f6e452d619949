#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; cd /tmp
for cfg in "P=1024" "P=256" "P=512" "P=2048x" "T=1"; do
  unset TKV_AMQ_PART_WGS TKV_AMQ_TILE1024
  case $cfg in
    P=1024) export TKV_AMQ_PART_WGS=1024;;
    P=256) export TKV_AMQ_PART_WGS=256;;
    P=512) export TKV_AMQ_PART_WGS=512;;
    P=2048x) export TKV_AMQ_PART_WGS=128;;
    T=1) export TKV_AMQ_TILE1024=1;;
  esac
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/exp_mono_$cfg -o run --output-format csv -- python3 $R/bench.py --workload bloom10mono --steps 5 --warmup 1 --no-cpu-baseline --ramp-ms 0 > $R/gpurun_out/exp_mono_$cfg.log 2>&1 || exit 1
done
