#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -q -m gpu -x > gpurun_out/kt7.log 2>&1 || { echo KT_FAIL; grep -E "Error|assert|FAILED|passed|failed" gpurun_out/kt7.log | tail -20; exit 1; }
tail -1 gpurun_out/kt7.log
timeout -k 10 300 python tools/attn_bench.py > gpurun_out/attn_bench7.jsonl 2>&1 || { echo AB_FAIL; tail -5 gpurun_out/attn_bench7.jsonl; exit 1; }
cat gpurun_out/attn_bench7.jsonl | grep '^{'
for b in 32 64; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --batch-per-gpu $b > gpurun_out/bench7_b$b.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/bench7_b$b.log; exit 1; }
  tail -1 gpurun_out/bench7_b$b.log | cut -c1-200
done
