#!/bin/bash
# tile kernel pieces of 64*V records: bloom10mono kernels and config 5 at 1B keys per library
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04/${TAG:-tilev}
mkdir -p $O
for L in main $LIBS; do
  n=$(basename $L .so)
  if [ $L = main ]; then unset TKV_AMQ_LIB; else export TKV_AMQ_LIB=$L; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$n -o p --output-format csv -- \
      python -u bench.py --workload bloom10mono --steps 20 --no-e2e --no-cpu-baseline > $O/mono_$n.log 2>&1 || exit 4
  echo "## $n"; python3 tools/kstats.py $O/prof_$n | grep "bloom_"; grep -o '"value": [0-9.]*\|"verified": [a-z]*' $O/mono_$n.log | head -2
  timeout -k 10 300 python -u bench.py --workload bloom12hash --total-keys 1000000000 --steps 5 --no-cpu-baseline --no-verify > $O/c5_$n.log 2>&1 || exit 5
  grep -o '"value": [0-9.]*' $O/c5_$n.log | head -1
done
