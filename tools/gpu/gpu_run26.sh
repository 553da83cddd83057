#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/ -q -m gpu -x > gpurun_out/gputests26.log 2>&1 || { echo GT_FAIL; grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/gputests26.log | tail -20; exit 1; }
tail -1 gpurun_out/gputests26.log
timeout -k 10 300 python tools/attn_bench.py > gpurun_out/attn26.jsonl 2>&1 || { echo AB_FAIL; tail -5 gpurun_out/attn26.jsonl; exit 1; }
grep '^{' gpurun_out/attn26.jsonl | head -3 | cut -c1-200
for ms in 0 1 0; do
DLLM_ATTN_MASK_STREAM=$ms timeout -k 10 300 python bench.py > gpurun_out/bench26_$ms.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/bench26_$ms.log; exit 1; }
echo "mask_stream=$ms $(tail -1 gpurun_out/bench26_$ms.log | cut -c1-200)"
done
