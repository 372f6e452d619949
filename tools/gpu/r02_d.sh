#!/bin/bash
# VQF iteration: GPU tests (VQF-heavy files first), small-batch curve, full vqf12 bench line
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/${O:-r02_d}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_robustness.py tests/test_gpu_pages_metrics.py tests/test_gpu_scale.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 2; }
tail -2 $O/t.log
timeout -k 10 300 python tools/small_batch.py --kind 1 --leaves 1,8,64,256,1024,2048,6104 > $O/curve_k1.log 2>&1 || exit 3
cat $O/curve_k1.log | grep kind
timeout -k 10 300 python bench.py --workload vqf12 --no-e2e --no-cpu-baseline > $O/b.log 2>&1 || exit 4
python -c "import json;d=json.loads(open('$O/b.log').read().strip().splitlines()[-1]);print(d['value'], d['roofline']['kernel_ms'], d['verified'], [(r['leaves'], r['ms'], r['mkeys_s']) for r in d.get('batch_sweep') or []])"
