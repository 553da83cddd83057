#!/bin/bash
# Long-sequence path after block-size-by-rows (8K blocks when batch x heads < 32) and conversion-free accumulation.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/p62
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "chunked or context_parallel or ring_attention" --timeout 200 --timeout-method thread > gpurun_out/t62.log 2>&1 || { echo T_FAIL; grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/t62.log | tail -30; exit 1; }
tail -1 gpurun_out/t62.log
for S in 16384 32768; do
  timeout -k 10 400 python bench.py --batch-per-gpu 1 --src-len $S --steps 5 --warmup 2 > gpurun_out/b62_$S.log 2>&1 || { echo B_FAIL; tail -20 gpurun_out/b62_$S.log; exit 1; }
  tail -1 gpurun_out/b62_$S.log | cut -c1-200
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/p62 -o run -- python bench.py --batch-per-gpu 1 --src-len 32768 --steps 2 --warmup 1 > gpurun_out/p62/log.txt 2>&1 || { echo P_FAIL; tail -20 gpurun_out/p62/log.txt; exit 1; }
python tools/prof_summary.py gpurun_out/p62/run_results.db 3 > gpurun_out/p62/summary.txt
rm -f gpurun_out/p62/run_results.db
head -8 gpurun_out/p62/summary.txt
