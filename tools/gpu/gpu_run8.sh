#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof8 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --batch-per-gpu 64 > $GRAFT_REPO_ROOT/gpurun_out/prof8.log 2>&1 || { echo PROF_FAIL; tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof8.log; exit 1; }
rm -f $GRAFT_REPO_ROOT/gpurun_out/prof8/run_kernel_trace.csv
python3 $GRAFT_REPO_ROOT/tools/prof_summary.py $GRAFT_REPO_ROOT/gpurun_out/prof8/run_kernel_stats.csv 7 | head -60
