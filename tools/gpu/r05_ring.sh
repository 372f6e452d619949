#!/bin/bash
# vqf_ring_place with its waves-per-SIMD stated (78 instead of 95 VGPRs): small VQF batches, A/B
set -o pipefail
O=gpurun_out/r05/ring; mkdir -p $O
export PYTHONUNBUFFERED=1
X="TKV_AMQ_EXPERIMENT=1 TKV_AMQ_LIB=$PWD/turtle_kv_amd/exp_head.so"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "vqf" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  && tail -2 $O/tests.log \
  && timeout -k 10 300 python -u tools/small_batch.py --kind 1 --leaves 1,64,256,512 > $O/new.log 2>&1 \
  && env $X timeout -k 10 300 python -u tools/small_batch.py --kind 1 --leaves 1,64,256,512 > $O/head.log 2>&1 \
  && timeout -k 10 300 python -u tools/small_batch.py --kind 1 --leaves 1,64,256,512 > $O/new2.log 2>&1
rc=$?; echo "rc=$rc"; paste <(grep -v amdgpu $O/head.log) <(grep -v amdgpu $O/new.log) <(grep -v amdgpu $O/new2.log); exit $rc
