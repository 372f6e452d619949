#!/bin/bash
# Monolithic Bloom experiments: parity under each library, then per-kernel rocprof stats.
#   LIBS="exp0 exp33" ./tools/gpu/mono_ab.sh
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/mono; mkdir -p $O; export TMPDIR=/tmp
for l in ${LIBS:-exp0}; do
  TKV_AMQ_LIB=$R/tools/exp/libtkv_amq_$l.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu \
    -k "monolithic" --timeout 120 --timeout-method thread > $O/tests_$l.log 2>&1 || exit 2
done
cd /tmp
for l in ${LIBS:-exp0}; do
  TKV_AMQ_LIB=$R/tools/exp/libtkv_amq_$l.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$l -o run --output-format csv -- python3 $R/bench.py --workload bloom10mono --no-cpu-baseline --no-e2e --steps 10 > $O/bench_$l.log 2>&1 || exit 3
done
