#!/bin/bash
# VQF small batches of variable-length keys: located keys (in-tree) vs the producers hashing ($LIBS)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04/${TAG:-varloc}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fuzz.py -k "vqf or VQF or fuzz" > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit 2
for L in main $LIBS; do
  n=$(basename $L .so)
  if [ $L = main ]; then unset TKV_AMQ_LIB; else export TKV_AMQ_LIB=$L; fi
  for KB in ${KBS:-0 20 16}; do
    timeout -k 10 300 python -u tools/small_batch.py --kind 1 --key-bytes $KB --leaves ${LEAVES:-1,8,64,256,512} --reps 50 > $O/small_${n}_$KB.log 2>&1 || exit 3
    echo "## $n key-bytes $KB"; grep median $O/small_${n}_$KB.log
  done
done
