#!/bin/bash
# round 4 final check: smoke(), the bench tests, the default bench line
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04/${TAG:-final}
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u -m pytest -q --timeout 600 --timeout-method thread tests/test_gpu_bench.py > $O/bench_tests.log 2>&1; rc=$?
echo "bench tests rc=$rc"; tail -2 $O/bench_tests.log; [ $rc -gt 1 ] && exit 3
timeout -k 10 300 python -u bench.py > $O/bench_default.log 2>&1 || exit 4
tail -1 $O/bench_default.log | cut -c1-400
