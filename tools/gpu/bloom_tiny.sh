set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/nows
timeout -k 10 200 python tools/small_batch.py --kind 0 --leaves 1,2,4,8,16,32,64,128 > gpurun_out/nows/ws.log 2>&1 || exit 2
timeout -k 10 200 python tools/small_batch.py --kind 0 --leaves 1,2,4,8,16,32,64,128 --no-ws > gpurun_out/nows/nows.log 2>&1 || exit 3
grep kind gpurun_out/nows/ws.log gpurun_out/nows/nows.log
