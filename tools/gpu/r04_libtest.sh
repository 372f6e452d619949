#!/bin/bash
# run one pytest selection under the in-tree library and each library in $LIBS
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04/${TAG:-libtest}
mkdir -p $O
for L in main $LIBS; do
  n=$(basename $L .so)
  if [ $L = main ]; then unset TKV_AMQ_LIB; else export TKV_AMQ_LIB=$L; fi
  timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread $TESTS -k "$K" > $O/t_$n.log 2>&1
  rc=$?
  echo "## $n rc=$rc"; tail -3 $O/t_$n.log
  if [ $rc -gt 1 ]; then exit 3; fi
done
