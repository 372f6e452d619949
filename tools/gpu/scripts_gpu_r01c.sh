#!/bin/bash
# round-1 GPU measurement script (run via gpurun); every GPU step has its own time limit
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 400 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 || exit 2
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_bloom10.log 2>&1 || exit 3
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --workload vqf12 --no-e2e > gpurun_out/bench_vqf12.log 2>&1 || exit 4
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --workload probe10 --no-cpu-baseline > gpurun_out/bench_probe10.log 2>&1 || exit 5
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $R/gpurun_out/prof_vqf12 -o run --output-format csv -- python3 $R/bench.py --workload vqf12 --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > $R/gpurun_out/prof_vqf12.log 2>&1 || exit 6
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc_sq -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $R/gpurun_out/pmc_sq.log 2>&1 || exit 7
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc_sq_vqf -o run --output-format csv -- python3 $R/bench.py --workload vqf12 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $R/gpurun_out/pmc_sq_vqf.log 2>&1 || exit 8
