#!/bin/bash
# quick iteration: the hash-shard tests, config 5 at 1B (kernel trace), bloom10mono
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r05/${TAG:-iter}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_hash_shard.py tests/test_gpu_parity.py -k "hash or shard or pipelined or route or mono or large or duplicate or range" -x -q --timeout 300 --timeout-method thread > $O/hash_shard.log 2>&1 || { tail -30 $O/hash_shard.log; exit 2; }
tail -1 $O/hash_shard.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o run --output-format csv -- python3 $R/bench.py --workload bloom12hash --total-keys 1000000000 --steps 10 --no-cpu-baseline --no-e2e > $O/c5.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_mono -o run --output-format csv -- python3 $R/bench.py --workload bloom10mono --no-cpu-baseline --no-e2e > $O/mono.log 2>&1 || exit 4
timeout -k 10 300 python3 $R/bench.py --workload bloom10monok24 --no-cpu-baseline --no-e2e > $O/monok24.log 2>&1 || exit 5
python3 $R/tools/kstats.py $O/prof_c5 $O/prof_mono
python3 - <<PY
import json
for w in ("c5", "mono", "monok24"):
    d = json.loads([l for l in open("$O/" + w + ".log") if l.startswith("{")][-1])
    print(w, d["value"], d["ms_per_step"], d["verified"], d.get("step_breakdown_rank0_ms"))
PY
