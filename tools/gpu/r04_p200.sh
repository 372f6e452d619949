#!/bin/bash
# 200-tile routed parts: mono + hash-range parity tests, config 5 at 1B keys (verified), profile
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04/${TAG:-p200}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_hash_shard.py tests/test_gpu_nccl.py -k "monolithic or hash or nccl or exchange" > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 $O/tests.log; [ $rc -ne 0 ] && exit 3
timeout -k 10 400 python -u bench.py --workload bloom12hash --total-keys 1000000000 --steps 10 --warmup 3 > $O/config5_n1.log 2>&1 || exit 4
grep -o '"value": [0-9.]*\|"verified": [a-z]*' $O/config5_n1.log | head -2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o p --output-format csv -- \
    python -u bench.py --workload bloom12hash --total-keys 1000000000 --steps 3 --warmup 1 --no-verify --no-cpu-baseline > $O/c5prof.log 2>&1 || exit 5
python3 tools/kstats.py $O/prof_c5 | grep "tkv::"
