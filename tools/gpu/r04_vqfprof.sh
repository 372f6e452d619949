#!/bin/bash
# kernel durations of the small-batch VQF build (rocprofv3 kernel trace), lone leaf and 64 leaves
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04/${TAG:-vqfprof}
mkdir -p $O
for Lv in ${LEAVES:-1 64 256}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof$Lv -o p --output-format csv -- \
      python tools/small_batch.py --kind 1 --leaves $Lv --reps 50 > $O/prof$Lv.log 2>&1 || exit 5
  echo "## leaves $Lv"; grep median $O/prof$Lv.log; python3 tools/kstats.py $O/prof$Lv | grep -v "gen_keys\|fill\|elementwise\|sort\|Kernel"
done
