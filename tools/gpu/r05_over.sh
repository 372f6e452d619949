#!/bin/bash
set -o pipefail
O=gpurun_out/r05/over; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_window.py tests/test_gpu_fuzz.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 3; }; tail -3 $O/tests.log
timeout -k 10 300 python -u tools/oversize_batch.py > $O/timing.log 2>&1 || { echo "timing failed"; tail -30 $O/timing.log; exit 3; }; cat $O/timing.log | grep -v amdgpu.ids
