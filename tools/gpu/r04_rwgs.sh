#!/bin/bash
# route workgroups (kRouteMaxWgs) per library ($LIBS): config 5 at 1B keys, route kernel times
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04/${TAG:-rwgs}
mkdir -p $O
for L in main $LIBS; do
  n=$(basename $L .so)
  if [ $L = main ]; then unset TKV_AMQ_LIB; else export TKV_AMQ_LIB=$L; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$n -o p --output-format csv -- \
      python -u bench.py --workload bloom12hash --total-keys 1000000000 --steps 5 --warmup 2 --no-cpu-baseline > $O/c5_$n.log 2>&1 || exit 4
  echo "## $n"; python3 tools/kstats.py $O/prof_$n | grep "route_\|bloom_part\|bloom_tile"; grep -o '"value": [0-9.]*\|"verified": [a-z]*' $O/c5_$n.log | head -2
  if [ $L != main ]; then
    timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_hash_shard.py tests/test_gpu_nccl.py -k "monolithic or hash or nccl or exchange or route" > $O/t_$n.log 2>&1; rc=$?
    echo "tests rc=$rc"; tail -1 $O/t_$n.log; [ $rc -ne 0 ] && exit 3
  fi
done
