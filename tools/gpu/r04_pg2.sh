cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04/pg2
for i in 1 2; do
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_bench.py -k "pipelined_gather_gloo" > gpurun_out/r04/pg2/run$i.log 2>&1; rc=$?
echo "run $i rc=$rc"; tail -2 gpurun_out/r04/pg2/run$i.log; [ $rc -gt 1 ] && exit 3
done
timeout -k 10 600 python -u -m pytest -q --timeout 500 --timeout-method thread tests/test_gpu_bench.py -k "probe_full_size" > gpurun_out/r04/pg2/probe.log 2>&1; echo "probe rc=$?"; tail -2 gpurun_out/r04/pg2/probe.log
