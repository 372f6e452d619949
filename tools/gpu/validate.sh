#!/bin/bash
# GPU tests, smoke, the default bench line (with the end-to-end legs); outputs in gpurun_out/$O
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=gpurun_out/${O:-val}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 2
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 3
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || exit 4
tail -n 1 $O/bench.log
