#!/bin/bash
# config 5 (1B keys, Bloom @12, hash-range on one GPU) with TILES tiles per routed part
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04/${TAG:-ptiles}
mkdir -p $O
for T in ${TILES:-1600 800 400 200}; do
  timeout -k 10 300 python -u tools/exp_part_tiles.py $T --workload bloom12hash --total-keys 1000000000 --steps 5 --warmup 2 --no-verify --no-cpu-baseline > $O/pt_$T.log 2>&1 || exit 2
  echo "tiles $T $(grep -o '"value": [0-9.]*' $O/pt_$T.log) $(grep -o 'in [0-9]* part(s)' $O/pt_$T.log)"
done
