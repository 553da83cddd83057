#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for pipe in 0 1; do
DLLM_ATTN_FWD_PIPE=$pipe timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x -k "attention" > gpurun_out/gputests16_$pipe.log 2>&1 || { echo GT_FAIL; grep -E "Error|assert|FAILED|passed|failed" gpurun_out/gputests16_$pipe.log | tail -20; exit 1; }
tail -1 gpurun_out/gputests16_$pipe.log
DLLM_ATTN_FWD_PIPE=$pipe timeout -k 10 300 python tools/attn_bench.py > gpurun_out/attn16_$pipe.jsonl 2>&1 || { echo AB_FAIL; tail -5 gpurun_out/attn16_$pipe.jsonl; exit 1; }
echo pipe=$pipe; grep '^{' gpurun_out/attn16_$pipe.jsonl | cut -c1-200
done
