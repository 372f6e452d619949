#!/bin/bash
# round 5, first GPU call: GPU suite, VQF repeatability stress (2 processes on the GPU), the
# default bench line (whole-output verification) and the VQF line.
set -o pipefail
O=gpurun_out/r05/a
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 3; }
tail -3 $O/gpu_tests.log
timeout -k 10 400 python -u tools/vqf_stress.py --iters 40 --procs 2 > $O/vqf_stress.log 2>&1 || { echo "stress failed"; tail -30 $O/vqf_stress.log; exit 3; }
tail -4 $O/vqf_stress.log
timeout -k 10 300 python -u bench.py > $O/bench_bloom10.log 2>&1 || exit 3
timeout -k 10 300 python -u bench.py --workload vqf12 > $O/bench_vqf12.log 2>&1 || exit 4
python - <<'PY'
import json
for w in ("bloom10", "vqf12"):
    d = json.loads(open(f"gpurun_out/r05/a/bench_{w}.log").read().strip().splitlines()[-1])
    print(w, d["value"], d["verified"], {k: d["verify"].get(k) for k in ("leaves_checked", "of_leaves", "keys_equal_oracle", "seconds")})
PY
