#!/bin/bash
# round 5: the one-pass route / pipelined hash-range form first (new kernels), then the GPU
# suite, the VQF repeatability stress, and the bench lines (default, vqf12, config 5 at 1B)
set -o pipefail
O=gpurun_out/r05/b
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_hash_shard.py -x -v --timeout 300 --timeout-method thread > $O/hash_shard.log 2>&1 || { tail -40 $O/hash_shard.log; exit 2; }
tail -2 $O/hash_shard.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 3; }; tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 3
timeout -k 10 400 python -u tools/vqf_stress.py --iters 30 --procs 2 > $O/vqf_stress.log 2>&1 || { echo "stress failed"; tail -30 $O/vqf_stress.log; exit 3; }; tail -3 $O/vqf_stress.log
timeout -k 10 300 python -u bench.py > $O/bench_bloom10.log 2>&1 || exit 4
timeout -k 10 300 python -u bench.py --workload vqf12 > $O/bench_vqf12.log 2>&1 || exit 5
timeout -k 10 400 python -u bench.py --workload bloom12hash --total-keys 1000000000 --steps 10 > $O/bench_c5_1B.log 2>&1 || exit 6
python - <<'PY'
import json
for w in ("bloom10", "vqf12", "c5_1B"):
    d = json.loads(open(f"gpurun_out/r05/b/bench_{w}.log").read().strip().splitlines()[-1])
    v = d.get("verify") or {}
    print(w, d["value"], d["ms_per_step"], d["verified"], {k: v.get(k) for k in ("leaves_checked", "of_leaves", "keys_equal_oracle", "seconds", "equal_to_oracle")}, d.get("step_breakdown_rank0_ms"))
PY
