#!/bin/bash
# round 4: time bench.py --workload ${W:-bloom10mono} under each library in $LIBS (kernel trace),
# the in-tree build first (with its parity tests)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04/${TAG:-libs}
mkdir -p $O
W=${W:-bloom10mono}
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py -k "monolithic and not large" > $O/tests.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_main -o p --output-format csv -- \
    python -u bench.py --workload $W --steps 20 --no-e2e --no-cpu-baseline > $O/bench_main.log 2>&1 || exit 3
for L in $LIBS; do
  n=$(basename $L .so)
  TKV_AMQ_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$n -o p --output-format csv -- \
      python -u bench.py --workload $W --steps 20 --no-e2e --no-cpu-baseline --no-verify > $O/bench_$n.log 2>&1 || exit 4
done
echo done
