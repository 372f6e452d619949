#!/bin/bash
# VQF probe with its per-lookup test inlined: parity, then A/B vs the previous library
set -o pipefail
O=gpurun_out/r05/vprobe; mkdir -p $O
export PYTHONUNBUFFERED=1
X="TKV_AMQ_EXPERIMENT=1 TKV_AMQ_LIB=$PWD/turtle_kv_amd/exp_head.so"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pages_metrics.py -x -q -k "probe or query or reject or metrics" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  && tail -2 $O/tests.log \
  && timeout -k 10 300 python -u bench.py --workload probe_vqf12 --no-e2e --no-cpu-baseline > $O/new.log 2>&1 \
  && env $X timeout -k 10 300 python -u bench.py --experiment-lib --workload probe_vqf12 --no-e2e --no-cpu-baseline > $O/head.log 2>&1 \
  && timeout -k 10 300 python -u bench.py --workload probe_vqf12 --no-e2e --no-cpu-baseline > $O/new2.log 2>&1
rc=$?; echo "rc=$rc"
for f in $O/new.log $O/head.log $O/new2.log; do grep '^{' $f | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$(basename $f)', d['value'], d['ms_per_step'], d.get('verified'))"; done
exit $rc
