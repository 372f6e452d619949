#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 120 ./tools/ubench_valu > gpurun_out/ubench_valu.log 2>&1 || exit 1
timeout -k 10 400 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 || exit 2
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_bloom10.log 2>&1 || exit 3
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $R/gpurun_out/prof_vqf12 -o run --output-format csv -- python3 $R/bench.py --workload vqf12 --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > $R/gpurun_out/prof_vqf12.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $R/gpurun_out/prof_bloom10 -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $R/gpurun_out/prof_bloom10.log 2>&1 || exit 5
timeout -k 10 120 rocprofv3 -L > $R/gpurun_out/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $R/gpurun_out/pmc_fetch.log 2>&1 || exit 6
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $R/gpurun_out/pmc_write.log 2>&1 || exit 7
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc_sq -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $R/gpurun_out/pmc_sq.log 2>&1 || exit 8
