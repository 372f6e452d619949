#!/bin/bash
# hash-range sharding: GPU tests (gloo ranks, RCCL world 1), then config 5 under RCCL world 1
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04/hs
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_hash_shard.py tests/test_gpu_nccl.py tests/test_gpu_bench.py -k "hash or nccl" > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit 2
PARTS=rccl1 TAG=config5 bash tools/gpu/r04_config5.sh
