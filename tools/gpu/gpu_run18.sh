#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/ -q -m gpu -x > gpurun_out/gputests18.log 2>&1 || { echo GT_FAIL; grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/gputests18.log | tail -20; exit 1; }
tail -1 gpurun_out/gputests18.log
timeout -k 10 300 python tools/attn_bench.py > gpurun_out/attn18.jsonl 2>&1 || { echo AB_FAIL; tail -5 gpurun_out/attn18.jsonl; exit 1; }
grep '^{' gpurun_out/attn18.jsonl | cut -c1-200
timeout -k 10 300 python bench.py > gpurun_out/bench18.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/bench18.log; exit 1; }
tail -1 gpurun_out/bench18.log | cut -c1-220
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof18b -o run --output-format csv -- python3 $R/bench.py --model bart-large --batch-per-gpu 32 --steps 5 --warmup 2 > $R/gpurun_out/prof18b.log 2>&1 || { echo PROF_FAIL; tail -20 $R/gpurun_out/prof18b.log; exit 1; }
rm -f $R/gpurun_out/prof18b/run_kernel_trace.csv
python3 $R/tools/prof_summary.py $R/gpurun_out/prof18b/run_kernel_stats.csv 7 > $R/gpurun_out/prof18b_summary.txt; head -50 $R/gpurun_out/prof18b_summary.txt
