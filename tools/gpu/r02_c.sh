#!/bin/bash
# GPU tests + one bench line without the end-to-end legs (iteration loop); gpurun_out/$O
set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/${O:-r02_c}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 2; }
tail -2 $O/t.log
timeout -k 10 300 python bench.py --no-e2e --no-cpu-baseline --sweep ${BENCH_ARGS} > $O/b.log 2>&1 || exit 3
python -c "import json;d=json.loads(open('$O/b.log').read().strip().splitlines()[-1]);print(d['value'], d['roofline']['kernel_ms'], [(r['leaves'], r['ms'], r['mkeys_s']) for r in d.get('batch_sweep') or []])"
