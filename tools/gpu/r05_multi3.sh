#!/bin/bash
# multi-leaf launches of up to 40 leaves (compact kernel argument) vs the previous library
set -o pipefail
O=gpurun_out/r05/multi3; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q -k "oversize" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  && tail -2 $O/tests.log \
  && timeout -k 10 300 python -u tools/oversize_batch.py > $O/new.log 2>&1 \
  && TKV_AMQ_EXPERIMENT=1 TKV_AMQ_LIB=$PWD/turtle_kv_amd/exp_head.so timeout -k 10 300 python -u tools/oversize_batch.py > $O/head.log 2>&1 \
  && timeout -k 10 300 python -u tools/oversize_batch.py > $O/new2.log 2>&1
echo "rc=$?"
paste <(grep keys $O/head.log) <(grep keys $O/new.log | sed 's/.*keys, //') <(grep keys $O/new2.log | sed 's/.*keys, //')
