#!/bin/bash
# single filters around the window / tiled threshold: the library vs an experiment build with kWinMonoMax = 1
set -o pipefail
O=gpurun_out/r05/winmono; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/single_filter.py > $O/main.log 2>&1 \
  && TKV_AMQ_EXPERIMENT=1 TKV_AMQ_LIB=$PWD/turtle_kv_amd/exp_winmono.so timeout -k 10 300 python -u tools/single_filter.py > $O/mono.log 2>&1
echo "rc=$?"
paste <(grep bpk $O/main.log) <(grep bpk $O/mono.log | sed 's/bpk [0-9]* n [0-9]*: [0-9]* windows,//')
