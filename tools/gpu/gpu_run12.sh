#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 12 600 python -m pytest tests/ -q -m gpu -x > gpurun_out/gputests12.log 2>&1 || { echo GT_FAIL; grep -E "Error|assert|FAILED|passed|failed" gpurun_out/gputests12.log | tail -20; exit 1; }
tail -1 gpurun_out/gputests12.log
for b in 64 32; do
  timeout -k 12 300 python bench.py --steps 12 --warmup 3 --batch-per-gpu $b > gpurun_out/bench12_b$b.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/bench12_b$b.log; exit 1; }
  tail -1 gpurun_out/bench12_b$b.log | cut -c1-200
done
cd /tmp && timeout -k 12 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof12 -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --batch-per-gpu 64 > $R/gpurun_out/prof12.log 2>&1 || { echo PROF_FAIL; tail -20 $R/gpurun_out/prof12.log; exit 1; }
rm -f $R/gpurun_out/prof12/run_kernel_trace.csv
python3 $R/tools/prof_summary.py $R/gpurun_out/prof12/run_kernel_stats.csv 7 > $R/gpurun_out/prof12_summary.txt; head -45 $R/gpurun_out/prof12_summary.txt
