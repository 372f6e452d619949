#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05/diag
timeout -k 10 300 python -u tools/diag_route_blocks.py > gpurun_out/r05/diag/route_blocks.log 2>&1 || { echo "failed"; tail -30 gpurun_out/r05/diag/route_blocks.log; exit 3; }
cat gpurun_out/r05/diag/route_blocks.log | tail -60
