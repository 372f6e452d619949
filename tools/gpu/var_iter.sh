#!/bin/bash
# variable-length key iteration: parity tests, bench lines, VALU per key
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${O:-var}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_window.py tests/test_cpp_mirror.py -x -v -k "${K:-variable or var or fuzz or mirror}" -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 2; }
tail -2 $O/tests.log
for W in ${WS:-bloom10var vqf12var}; do
  timeout -k 10 300 python bench.py --workload $W --no-e2e --no-cpu-baseline > $O/bench_$W.log 2>&1 || exit 3
  python3 -c "import json,sys; d=json.loads(open('$O/bench_$W.log').read().strip().splitlines()[-1]); print('$W', d['value'], d['ms_per_step'], d.get('verified'))"
done
LENS="${LENS:-8,32 24,25}" O=${O#gpurun_out/}_pmc bash tools/gpu/pmc_var.sh
