#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x -k "attention" > gpurun_out/gputests24a.log 2>&1 || { echo GT_FAIL; grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/gputests24a.log | tail -20; exit 1; }
tail -1 gpurun_out/gputests24a.log
timeout -k 10 600 python -m pytest tests/ -q -m gpu -x > gpurun_out/gputests24.log 2>&1 || { echo GT_FAIL; grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/gputests24.log | tail -20; exit 1; }
tail -1 gpurun_out/gputests24.log
for bg in atomic shear; do
DLLM_ATTN_BGRAD=$bg timeout -k 10 300 python tools/attn_bench.py > gpurun_out/attn24_$bg.jsonl 2>&1 || { echo AB_FAIL; tail -5 gpurun_out/attn24_$bg.jsonl; exit 1; }
echo "bgrad=$bg"; grep '^{' gpurun_out/attn24_$bg.jsonl | cut -c1-200
done
for v in "0 atomic" "1 atomic" "0 shear"; do
set -- $v
DLLM_ATTN_MASK_STREAM=$1 DLLM_ATTN_BGRAD=$2 timeout -k 10 300 python bench.py > gpurun_out/bench24_$1_$2.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/bench24_$1_$2.log; exit 1; }
echo "mask_stream=$1 bgrad=$2 $(tail -1 gpurun_out/bench24_$1_$2.log | cut -c1-200)"
done
