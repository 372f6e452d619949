#!/bin/bash
# 24-byte-key partition with the store table: parity, then A/B bench vs the previous library
set -o pipefail
O=gpurun_out/r05/k24tbl; mkdir -p $O
export PYTHONUNBUFFERED=1
X="TKV_AMQ_EXPERIMENT=1 TKV_AMQ_LIB=$PWD/turtle_kv_amd/exp_head.so"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_window.py tests/test_gpu_hash_shard.py -x -q -k "k24 or 24 or oversize or monolithic" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  && tail -2 $O/tests.log \
  && timeout -k 10 300 python -u bench.py --workload bloom10monok24 --no-e2e --no-cpu-baseline > $O/k24_new.log 2>&1 \
  && env $X timeout -k 10 300 python -u bench.py --experiment-lib --workload bloom10monok24 --no-e2e --no-cpu-baseline > $O/k24_head.log 2>&1 \
  && timeout -k 10 300 python -u bench.py --workload bloom10monok24 --no-e2e --no-cpu-baseline > $O/k24_new2.log 2>&1
rc=$?; echo "rc=$rc"
for f in $O/k24_*.log; do grep '^{' $f | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$(basename $f)', d['value'], d['ms_per_step'], d.get('verified'))"; done
exit $rc
