#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r05/${TAG:-vqfvar}; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "vqf" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 3; }; tail -3 $O/tests.log
[ $rc -eq 0 ] || exit 2
cd /tmp
for W in vqf12var vqf12; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$W -o run --output-format csv -- python3 $R/bench.py --workload $W --no-cpu-baseline --no-e2e > $O/$W.log 2>&1 || exit 3
done
python3 $R/tools/kstats.py $O/prof_vqf12var $O/prof_vqf12
for W in vqf12var vqf12; do grep '^{' $O/$W.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$W', d['value'], d['ms_per_step'], d['verified'], d['verify']['leaves_checked'], d['roofline']['kernel_ms'])"; done
