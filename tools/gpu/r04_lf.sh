#!/bin/bash
# partition experiment libraries ($LIBS): mono parity tests, bloom10mono kernels, config 5 at 1B
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04/${TAG:-lf}
mkdir -p $O
for L in main $LIBS; do
  n=$(basename $L .so)
  if [ $L = main ]; then unset TKV_AMQ_LIB; else export TKV_AMQ_LIB=$L; fi
  timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_hash_shard.py -k "monolithic or hash" > $O/t_$n.log 2>&1; rc=$?
  echo "## $n tests rc=$rc"; tail -1 $O/t_$n.log; [ $rc -gt 1 ] && exit 3
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$n -o p --output-format csv -- \
      python -u bench.py --workload bloom10mono --steps 20 --no-e2e --no-cpu-baseline --no-verify > $O/mono_$n.log 2>&1 || exit 4
  python3 tools/kstats.py $O/prof_$n | grep "bloom_"; grep -o '"value": [0-9.]*' $O/mono_$n.log | head -1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof1b_$n -o p --output-format csv -- \
      python -u bench.py --workload bloom12hash --total-keys 1000000000 --steps 5 --no-cpu-baseline --no-verify > $O/c5_$n.log 2>&1 || exit 5
  python3 tools/kstats.py $O/prof1b_$n | grep "bloom_\|route"; grep -o '"value": [0-9.]*' $O/c5_$n.log | head -1
done
