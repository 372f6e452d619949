#!/bin/bash
# tile-kernel variant: parity of the monolithic/oversize tests, oversize timings, bloom10mono line, kernel trace
set -o pipefail
O=gpurun_out/r05/${TAG:-multi2}; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_window.py -x -q -k "oversize or monolithic or window" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  && tail -2 $O/tests.log \
  && timeout -k 10 300 python -u tools/oversize_batch.py > $O/timing.log 2>&1 \
  && grep -v amdgpu.ids $O/timing.log \
  && timeout -k 10 300 python -u bench.py --workload bloom10mono --no-cpu-baseline --no-e2e > $O/mono.log 2>&1 \
  && grep '^{' $O/mono.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print("mono", d["value"], d["ms_per_step"], d["verified"])' \
  && export TMPDIR=/tmp \
  && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/oversize_batch.py > $O/prof.log 2>&1 \
  && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_mono -o run --output-format csv -- python3 bench.py --workload bloom10mono --no-cpu-baseline --no-e2e > $O/prof_mono.log 2>&1
echo "rc=$?"
