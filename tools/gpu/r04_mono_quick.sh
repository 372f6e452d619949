#!/bin/bash
# round 4: quick timing of the monolithic build (bench line + kernel trace), and the
# two-workgroups-per-CU partition experiment build (${EXP:-tools/exp/libtkv_amq_v8.so})
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04/${TAG:-q}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py -k "monolithic and not large" > $O/tests.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o p --output-format csv -- \
    python -u bench.py --workload bloom10mono --steps 20 --no-e2e --no-cpu-baseline > $O/bench_bloom10mono.log 2>&1 &&
if [ -f ${EXP:-tools/exp/libtkv_amq_v8.so} ]; then
  TKV_AMQ_LIB=${EXP:-tools/exp/libtkv_amq_v8.so} timeout -k 10 300 python -u -m pytest -x -q --timeout 300 \
      --timeout-method thread tests/test_gpu_parity.py -k "monolithic and not large" > $O/tests_exp.log 2>&1 &&
  TKV_AMQ_LIB=${EXP:-tools/exp/libtkv_amq_v8.so} timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_exp \
      -o p --output-format csv -- python -u bench.py --workload bloom10mono --steps 20 --no-e2e \
      --no-cpu-baseline > $O/bench_bloom10mono_exp.log 2>&1
fi
rc=$?
echo "exit $rc"
exit $rc
