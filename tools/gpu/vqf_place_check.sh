set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/p3; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 2
for rep in 1 2; do for l in head place3; do TKV_AMQ_LIB=$R/tools/exp/libtkv_amq_$l.so timeout -k 10 200 python bench.py --workload vqf12 --no-cpu-baseline --no-e2e --steps 10 > $O/vqf12_$l.log 2>&1 || exit 3; echo "$l $(tail -n 1 $O/vqf12_$l.log | python -c 'import json,sys; l=json.loads(sys.stdin.read()); print(l["value"], l["roofline"]["kernel_ms"])')"; done; done
cd /tmp
for pass in "fetch:FETCH_SIZE" "write:WRITE_SIZE" "sq:SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  name=${pass%%:*}; ctrs=${pass#*:}
  timeout -k 10 -s KILL 240 rocprofv3 --pmc $ctrs -d $O/pmc_vqf12_$name -o run --output-format csv -- python3 $R/bench.py --workload vqf12 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --ramp-ms 0 > $O/pmc_vqf12_$name.log 2>&1 || exit 4
done
