#!/bin/bash
# VQF iteration: the VQF parity / robustness tests, then the small-batch timings and kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${O:-vqf}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_robustness.py tests/test_gpu_pages_metrics.py tests/test_gpu_scale.py tests/test_gpu_graph.py -x -v -k "${K:-vqf or VQF or robust or status or workspace or overflow or graph or page}" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 2; }
tail -3 $O/tests.log
timeout -k 10 300 python tools/small_batch.py --kind 1 --leaves ${LEAVES:-1,8,64,256,512,768,1024,6104} --reps 50 2>&1 | grep -v amdgpu.ids > $O/timing.log || exit 3
cat $O/timing.log
cd /tmp && export TMPDIR=/tmp
for L in 1 64; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof$L -o p --output-format csv -- python $GRAFT_REPO_ROOT/tools/small_batch.py --kind 1 --leaves $L --reps 50 > $GRAFT_REPO_ROOT/$O/prof$L.log 2>&1 || exit 5
python3 - $GRAFT_REPO_ROOT/$O/prof$L/p_kernel_stats.csv $L <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'tkv' in r['Name'] or 'fill' in r['Name']:
        print(sys.argv[2], r['Name'][:48], r['Calls'], round(float(r['AverageNs'])/1000, 2), round(float(r['MinNs'])/1000, 2))
PY
done
