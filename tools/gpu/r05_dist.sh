#!/bin/bash
# config 5's pipelined step at its own size: 8 gloo ranks sharing the GPU (the multi-rank logic:
# route blocks -> all_to_all_single of equal splits -> part builds -> in-place round gathers),
# and one RCCL rank under torch.distributed.run; both verified whole against the oracle
set -o pipefail
O=gpurun_out/r05/dist; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u bench.py --gpus 8 --backend gloo --workload bloom12hash --total-keys 1000000000 --steps 1 --warmup 0 --ramp-ms 0 --no-cpu-baseline > $O/gloo8_c5_1B.log 2>&1 || { echo "gloo8 failed"; tail -30 $O/gloo8_c5_1B.log; exit 3; }; grep '^{' $O/gloo8_c5_1B.log | cut -c1-600
timeout -k 10 600 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --workload bloom12hash --total-keys 1000000000 --steps 10 > $O/rccl1_c5_1B.log 2>&1 || { echo "rccl1 failed"; tail -30 $O/rccl1_c5_1B.log; exit 3; }; grep '^{' $O/rccl1_c5_1B.log | cut -c1-600
