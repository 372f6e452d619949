#!/bin/bash
# VQF small-batch curve only (quick latency check)
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/${O:-r02_e}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "vqf" --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 2; }
tail -1 $O/t.log
timeout -k 10 300 python tools/small_batch.py --kind 1 --leaves ${CL:-1,64,256,1024,6104} > $O/curve_k1.log 2>&1 || exit 3
grep kind $O/curve_k1.log
