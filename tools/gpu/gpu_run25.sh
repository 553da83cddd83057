#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x -k "attention" > gpurun_out/gputests25a.log 2>&1 || { echo GT_FAIL; grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/gputests25a.log | tail -20; exit 1; }
tail -1 gpurun_out/gputests25a.log
DLLM_ATTN_DKDV_RING=1 timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x -k "attention" > gpurun_out/gputests25b.log 2>&1 || { echo GT_FAIL; grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/gputests25b.log | tail -20; exit 1; }
tail -1 gpurun_out/gputests25b.log
for ring in 0 1; do
DLLM_ATTN_DKDV_RING=$ring timeout -k 10 300 python tools/attn_bench.py > gpurun_out/attn25_$ring.jsonl 2>&1 || { echo AB_FAIL; tail -5 gpurun_out/attn25_$ring.jsonl; exit 1; }
echo "ring=$ring"; grep '^{' gpurun_out/attn25_$ring.jsonl | cut -c1-200
DLLM_ATTN_DKDV_RING=$ring timeout -k 10 300 python bench.py > gpurun_out/bench25_$ring.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/bench25_$ring.log; exit 1; }
echo "ring=$ring $(tail -1 gpurun_out/bench25_$ring.log | cut -c1-200)"
done
