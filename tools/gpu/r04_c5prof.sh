#!/bin/bash
# kernel statistics of the config-5 step at 1B keys on one GPU, and of the monolithic workloads
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04/${TAG:-c5prof}
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o p --output-format csv -- \
    python -u bench.py --workload bloom12hash --total-keys 1000000000 --steps 3 --warmup 1 --no-verify --no-cpu-baseline > $O/c5.log 2>&1 || exit 2
python3 tools/kstats.py $O/prof_c5 | grep "tkv::"; grep -o '"value": [0-9.]*' $O/c5.log
for W in bloom10monok24 bloom12hash; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$W -o p --output-format csv -- \
    python -u bench.py --workload $W --steps 10 --no-e2e --no-cpu-baseline > $O/$W.log 2>&1 || exit 3
python3 tools/kstats.py $O/prof_$W | grep "tkv::"; grep -o '"value": [0-9.]*\|"verified": [a-z]*' $O/$W.log
done
