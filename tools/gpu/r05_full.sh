#!/bin/bash
# whole GPU suite, smoke, then the single-filter and oversize timings
set -o pipefail
O=gpurun_out/r05/${TAG:-full}; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 \
  && tail -3 $O/gpu_tests.log \
  && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 \
  && tail -1 $O/smoke.log \
  && timeout -k 10 300 python -u tools/single_filter.py > $O/single.log 2>&1 \
  && timeout -k 10 300 python -u tools/oversize_batch.py > $O/oversize.log 2>&1 \
  && timeout -k 10 300 python -u tools/window_batch.py > $O/window_batch.log 2>&1 \
  && grep -hv amdgpu.ids $O/single.log $O/oversize.log $O/window_batch.log
rc=$?; echo "rc=$rc"; tail -5 $O/gpu_tests.log | grep -E "passed|failed|error" ; exit $rc
