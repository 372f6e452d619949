#!/bin/bash
# kernel-trace stats of one bench workload under several experiment libraries (LIBS, W)
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/${O:-proflibs}; mkdir -p $O
for l in ${LIBS:-cur}; do
  TKV_AMQ_LIB=$GRAFT_REPO_ROOT/tools/exp/libtkv_amq_$l.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$l -o run -- python bench.py --workload ${W:-bloom10mono} --no-cpu-baseline --no-e2e --no-verify --steps 20 > $O/$l.log 2>&1 || exit 3
  echo "== $l"; python3 -c "
import csv,glob
for r in csv.DictReader(open(glob.glob('$O/$l/**/run_kernel_stats.csv', recursive=True)[0])):
    if 'tkv::' in r['Name'] and 'gen_keys' not in r['Name']: print(r['Name'].split('(')[0][:40], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')"
done
