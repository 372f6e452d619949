#!/bin/bash
# round 4 batch: VQF ring-prefix parity under experiment libs, small-batch VQF timings, the
# looped tile kernel (parity + bloom10mono), pipelined all-gather bench tests, config 5 at N=1.
# A step that fails its tests (rc 1) does not stop the batch; anything worse (a fault, an abort,
# a time limit) ends it there.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04/${TAG:-batch}
mkdir -p $O
ok() { local rc=$1; if [ $rc -gt 1 ]; then echo "stop: rc=$rc at $2"; exit 3; fi; }
PT="python -u -m pytest -q --timeout 300 --timeout-method thread"
has() { [[ " ${PARTS:-vqf small tile gather leaf c5} " == *" $1 "* ]]; }
if has vqf; then
for L in main $VQFLIBS; do
  n=$(basename $L .so)
  if [ $L = main ]; then unset TKV_AMQ_LIB; else export TKV_AMQ_LIB=$L; fi
  timeout -k 10 300 $PT tests/test_gpu_parity.py -k "vqf_parity or ring_prefix or ring_place" > $O/vqf_$n.log 2>&1; rc=$?
  echo "## vqf $n rc=$rc"; tail -2 $O/vqf_$n.log; ok $rc vqf_$n
done
unset TKV_AMQ_LIB
fi
if has small; then
for L in main $VQFLIBS; do
  n=$(basename $L .so)
  if [ $L = main ]; then unset TKV_AMQ_LIB; else export TKV_AMQ_LIB=$L; fi
  timeout -k 10 300 python -u tools/small_batch.py --kind 1 --leaves 1,8,64,256,512 --reps 50 > $O/small_$n.log 2>&1; ok $? small_$n
  echo "## small $n"; grep -v amdgpu.ids $O/small_$n.log | tail -8
done
unset TKV_AMQ_LIB
fi
if has tile; then
for L in main $TILELIBS; do
  n=$(basename $L .so)
  if [ $L = main ]; then unset TKV_AMQ_LIB; else export TKV_AMQ_LIB=$L; fi
  timeout -k 10 400 $PT tests/test_gpu_parity.py tests/test_gpu_hash_shard.py -k "monolithic or hash" > $O/mono_$n.log 2>&1; rc=$?
  echo "## mono tests $n rc=$rc"; tail -2 $O/mono_$n.log; ok $rc mono_$n
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$n -o p --output-format csv -- \
      python -u bench.py --workload bloom10mono --steps 20 --no-e2e --no-cpu-baseline > $O/bench_mono_$n.log 2>&1; ok $? bench_$n
  python3 tools/kstats.py $O/prof_$n | grep -i "bloom\|value" ; grep -o '"value": [0-9.]*' $O/bench_mono_$n.log
done
unset TKV_AMQ_LIB
fi
if has gather; then
  timeout -k 10 600 $PT tests/test_gpu_bench.py -k "pipelined or host_legs or nccl_world1" > $O/gather_tests.log 2>&1; rc=$?
  echo "## gather tests rc=$rc"; tail -3 $O/gather_tests.log; ok $rc gather
  timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
      --master-port 29517 bench.py --gpus 1 --chunks 4 --steps 10 --no-cpu-baseline > $O/bench_chunks_rccl1.log 2>&1; ok $? chunks
  tail -1 $O/bench_chunks_rccl1.log | cut -c1-600
fi
if has leaf; then
  # per-leaf drop-in vs LeafBatcher from T host threads (tools/leaf_bench.cpp)
  B=$O/leaf_bench.txt; : > $B
  for kind in 0 1; do for t in 8 16; do for bt in 0 1; do
    timeout -k 10 60 ./tools/leaf_bench $t 2048 16384 $kind $bt >> $B 2>&1; ok $? leaf
  done; done; done
  cat $B
fi
if has c5; then
  timeout -k 10 600 python -u bench.py --workload bloom12hash --total-keys 1000000000 --steps 10 \
      --no-cpu-baseline > $O/bench_bloom12hash_1B_n1.log 2>&1; ok $? c5_n1
  tail -1 $O/bench_bloom12hash_1B_n1.log | cut -c1-900
fi
echo done
