#!/bin/bash
# multi-leaf oversize build: parity of every oversize test, then the batch timings and a kernel trace
set -o pipefail
O=gpurun_out/r05/multi; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -v -k "oversize or monolithic" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  && tail -3 $O/tests.log \
  && timeout -k 10 300 python -u tools/oversize_batch.py > $O/timing.log 2>&1 \
  && grep -v amdgpu.ids $O/timing.log \
  && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT \
  && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/oversize_batch.py > $O/prof.log 2>&1 \
  && find $O/prof -name "*kernel_stats.csv" -exec head -12 {} \;
echo "rc=$?"
tail -30 $O/tests.log | grep -E "PASS|FAIL|Error|error" | tail -20
