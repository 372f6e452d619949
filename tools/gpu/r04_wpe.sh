#!/bin/bash
# vqf12 under libraries built with different waves-per-EU bounds on vqf_decide ($LIBS)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04/${TAG:-wpe}
mkdir -p $O
for L in main $LIBS; do
  n=$(basename $L .so)
  if [ $L = main ]; then unset TKV_AMQ_LIB; else export TKV_AMQ_LIB=$L; fi
  timeout -k 10 300 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "vqf_parity or decide_paths or config1" > $O/t_$n.log 2>&1; rc=$?
  echo "## $n tests rc=$rc"; tail -1 $O/t_$n.log; [ $rc -gt 1 ] && exit 3
  for W in vqf12 vqf12var vqf12k24; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_${n}_$W -o p --output-format csv -- \
        python -u bench.py --workload $W --steps 20 --no-e2e --no-cpu-baseline > $O/bench_${n}_$W.log 2>&1 || exit 4
    echo "$n $W $(grep -o '"value": [0-9.]*' $O/bench_${n}_$W.log | head -1)"; python3 tools/kstats.py $O/prof_${n}_$W | grep "vqf_decide\|vqf_place"
  done
done
