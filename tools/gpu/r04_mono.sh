#!/bin/bash
# round 4: the monolithic / hash-range Bloom rebuild -- parity tests, bench lines, kernel trace
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py -k "monolithic" tests/test_gpu_hash_shard.py > $O/mono_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --workload bloom10mono --no-e2e --no-cpu-baseline > $O/bench_bloom10mono.log 2>&1 &&
timeout -k 10 300 python -u bench.py --workload bloom12hash --no-cpu-baseline > $O/bench_bloom12hash.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_mono -o prof -- \
    python -u bench.py --workload bloom10mono --steps 10 --no-e2e --no-cpu-baseline --no-verify > $O/prof_mono.log 2>&1
rc=$?
echo "exit $rc"
exit $rc
