#!/bin/bash
# one VALU PMC pass over a small_batch workload (args in $ARGS)
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/pmcv; cd /tmp; export TMPDIR=/tmp
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/pmcv/${TAG:-a} -o run --output-format csv -- python3 $R/tools/small_batch.py $ARGS > $R/gpurun_out/pmcv/${TAG:-a}.log 2>&1
