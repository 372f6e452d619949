#!/bin/bash
# Kernel experiments: build libtkv_amq variants with -DTKV_EXP=<n> (here, no GPU needed),
# then time them on the GPU box:  EXPS="0 1 2" W=vqf12 tools/exp_variants.sh run
# The experiment switches (TKV_EXP, TKV_STAGE_R, TKV_VQF_PROBE_BOTH) are not in the product
# source: tools/patches/kernel_experiments.patch adds them to a copy under tools/exp/src.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
EXPS=${EXPS:-0 1 2 3 4 5}
if [ "$1" != "run" ]; then
  mkdir -p $R/tools/exp/src/turtle_kv_amd/csrc
  cp $R/turtle_kv_amd/csrc/* $R/tools/exp/src/turtle_kv_amd/csrc/
  (cd $R/tools/exp/src && patch -s -p1 < $R/tools/patches/kernel_experiments.patch) || exit 1
  for e in $EXPS; do
    /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -shared -fPIC -DTKV_EXP=$e \
      -I$R/include -o $R/tools/exp/libtkv_amq_exp$e.so $R/tools/exp/src/turtle_kv_amd/csrc/tkv_amq_kernels.hip \
      $R/tools/exp/src/turtle_kv_amd/csrc/tkv_amq_stage.cpp &
  done
  wait
  exit 0
fi
cd $R; mkdir -p gpurun_out
for e in $EXPS; do
  TKV_AMQ_LIB=$R/tools/exp/libtkv_amq_exp$e.so timeout -k 10 200 python bench.py --workload ${W:-vqf12} \
    --no-cpu-baseline --no-e2e --steps 20 > gpurun_out/exp_$e.log 2>&1 || exit 3
  echo "exp $e: $(python -c "import json;l=json.loads(open('gpurun_out/exp_$e.log').read().strip().splitlines()[-1]);print(l['value'], l['roofline']['kernel_ms'])")"
done
