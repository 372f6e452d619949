#!/bin/bash
# round 4: BASELINE config 5 read literally at its own size -- one Bloom filter @12 bits/key
# over 1B 16-byte keys, hash-range sharded: N = 1 without a process group, N = 1 under
# torch.distributed.run (RCCL world 1: route -> all-to-all -> part builds), and the 8-rank
# rehearsal with gloo ranks sharing the one GPU.  Every line checks the filter against a
# one-GPU build and the oracle (header + 8 sampled tiles, every key hashed).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04/${TAG:-config5}
mkdir -p $O
PARTS=${PARTS:-n1 rccl1 gloo8}
has() { [[ " $PARTS " == *" $1 "* ]]; }
if has n1; then
  timeout -k 10 600 python -u bench.py --workload bloom12hash --total-keys 1000000000 --steps 10 \
      --no-cpu-baseline > $O/bench_bloom12hash_1B_n1.log 2>&1 || exit 2
fi
if has rccl1; then
  timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
      --master-addr 127.0.0.1 --master-port 29511 bench.py --workload bloom12hash \
      --total-keys 1000000000 --steps 5 --no-cpu-baseline > $O/bench_bloom12hash_1B_rccl1.log 2>&1 || exit 3
fi
if has gloo8; then
  timeout -k 10 1000 python -u bench.py --gpus 8 --backend gloo --workload bloom12hash \
      --total-keys 1000000000 --steps 1 --warmup 0 --ramp-ms 0 > $O/bench_bloom12hash_1B_gloo8.log 2>&1 || exit 4
fi
echo done
