#!/bin/bash
# VALU per key of the Bloom variable-length build by key-length mix (PMC SQ_INSTS_VALU pass)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/${O:-pmcvar}; mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for L in ${LENS:-8,32 24,25 16,17 8,9}; do
  n=${L/,/_}
  timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d $O/v_$n -o run --output-format csv -- python3 $R/tools/small_batch.py --kind ${KIND:-0} --key-bytes 0 --var-lens $L --leaves 6104 --reps 3 > $O/v_$n.log 2>&1 || exit 3
  python3 - $O/v_$n/run_counter_collection.csv $L <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float)); disp = collections.defaultdict(set)
for r in rows:
    k = r['Kernel_Name'][:60]
    agg[k][r['Counter_Name']] += float(r['Counter_Value']); disp[k].add(r['Dispatch_Id'])
keys = 6104 * 16384
for k, c in agg.items():
    if 'tkv' not in k: continue
    nd = len(disp[k])
    print(sys.argv[2], k, 'dispatches', nd, 'VALU/key %.1f' % (c['SQ_INSTS_VALU'] * 64 / keys / nd),
          'waves', c['SQ_WAVES'] / nd)
PY
done
