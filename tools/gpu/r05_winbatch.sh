#!/bin/bash
# batches of 5-16-window leaves: window path (previous library, experiment) vs the tiled multi-leaf build (library),
# then the parity tests of both paths
set -o pipefail
O=gpurun_out/r05/winbatch; mkdir -p $O
export PYTHONUNBUFFERED=1
TKV_AMQ_EXPERIMENT=1 TKV_AMQ_LIB=$PWD/turtle_kv_amd/exp_head.so timeout -k 10 400 python -u tools/window_batch.py > $O/window.log 2>&1 \
  && timeout -k 10 400 python -u tools/window_batch.py > $O/multi.log 2>&1 \
  && timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_window.py -x -q -k "oversize or monolithic or window" --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo "rc=$?"; tail -2 $O/tests.log
paste <(grep keys $O/window.log) <(grep keys $O/multi.log | sed 's/.*keys, //')
