#!/bin/bash
# round 4: VQF small batches with the located-key pre-pass and parallel prefix -- the ring
# parity tests, then small-batch timings (in-tree library, and each library in $LIBS)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04/${TAG:-vqfloc}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    -k "${K:-ring_prefix or ring_place or decide_paths or vqf_parity or unsorted or config1_sha}" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 2; }
tail -2 $O/tests.log
timeout -k 10 300 python -u tools/small_batch.py --kind 1 --leaves ${LEAVES:-1,8,64,256,512} --reps 50 > $O/timing_main.log 2>&1 || exit 3
grep -v amdgpu.ids $O/timing_main.log
for L in $LIBS; do
  n=$(basename $L .so)
  TKV_AMQ_LIB=$L timeout -k 10 300 python -u tools/small_batch.py --kind 1 --leaves ${LEAVES:-1,8,64,256,512} --reps 50 > $O/timing_$n.log 2>&1 || exit 4
  echo "## $n"; grep -v amdgpu.ids $O/timing_$n.log
done
for Lv in 1 64; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof$Lv -o p --output-format csv -- python tools/small_batch.py --kind 1 --leaves $Lv --reps 50 > $O/prof$Lv.log 2>&1 || exit 5
python3 tools/kstats.py $O/prof$Lv
done
echo done
