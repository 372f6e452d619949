#!/bin/bash
set -o pipefail
O=gpurun_out/r05/winbatch4; mkdir -p $O
export PYTHONUNBUFFERED=1
TKV_AMQ_EXPERIMENT=1 TKV_AMQ_LIB=$PWD/turtle_kv_amd/exp_head.so timeout -k 10 400 python -u tools/window_batch.py > $O/window.log 2>&1 \
  && timeout -k 10 400 python -u tools/window_batch.py > $O/multi.log 2>&1 \
  && TKV_AMQ_EXPERIMENT=1 TKV_AMQ_LIB=$PWD/turtle_kv_amd/exp_head.so timeout -k 10 300 python -u tools/oversize_batch.py > $O/over_head.log 2>&1 \
  && timeout -k 10 300 python -u tools/oversize_batch.py > $O/over_new.log 2>&1 \
  && timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_window.py -x -q -k "oversize or monolithic or window" --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo "rc=$?"; tail -2 $O/tests.log
paste <(grep keys $O/window.log) <(grep keys $O/multi.log | sed 's/.*keys, //')
paste <(grep keys $O/over_head.log) <(grep keys $O/over_new.log | sed 's/.*keys, //')
