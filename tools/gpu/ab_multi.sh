#!/bin/bash
# Product GPU tests, monolithic parity under experiment libraries, then A/B timings:
#   PAIRS="workload:lib,lib,... workload:lib,..."   (lib = tools/exp/libtkv_amq_<lib>.so)
#   MONO_LIBS="exp31 exp32"                          (monolithic parity tests under these libs)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/ab; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 2
for l in $MONO_LIBS; do
  TKV_AMQ_LIB=$R/tools/exp/libtkv_amq_$l.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu \
    -k "monolithic_partitioned or monolithic_duplicate" --timeout 120 --timeout-method thread > $O/mono_tests_$l.log 2>&1 || exit 3
done
for rep in 1 2; do
  for pair in $PAIRS; do
    W=${pair%%:*}; libs=${pair#*:}
    for l in ${libs//,/ }; do
      TKV_AMQ_LIB=$R/tools/exp/libtkv_amq_$l.so timeout -k 10 200 python bench.py --workload $W \
        --no-cpu-baseline --no-e2e --steps 10 > $O/${W}_$l.log 2>&1 || exit 4
      echo "$W $l: $(python -c "import json;l=json.loads(open('$O/${W}_$l.log').read().strip().splitlines()[-1]);print(l['value'], l['roofline']['kernel_ms'])")"
    done
  done
done
