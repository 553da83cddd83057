#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/ -q -m gpu -x > gpurun_out/gputests23.log 2>&1 || { echo GT_FAIL; grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/gputests23.log | tail -20; exit 1; }
tail -1 gpurun_out/gputests23.log
timeout -k 10 300 python tools/attn_bench.py > gpurun_out/attn23.jsonl 2>&1 || { echo AB_FAIL; tail -5 gpurun_out/attn23.jsonl; exit 1; }
grep '^{' gpurun_out/attn23.jsonl | head -2 | cut -c1-200
for ms in 0 1; do
DLLM_ATTN_MASK_STREAM=$ms timeout -k 10 300 python bench.py > gpurun_out/bench23_$ms.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/bench23_$ms.log; exit 1; }
echo "mask_stream=$ms $(tail -1 gpurun_out/bench23_$ms.log | cut -c1-200)"
done
for bg in shear atomic; do
DLLM_ATTN_BGRAD=$bg timeout -k 10 300 python tools/attn_bench.py > gpurun_out/attn23_$bg.jsonl 2>&1 || { echo AB_FAIL; tail -5 gpurun_out/attn23_$bg.jsonl; exit 1; }
echo "bgrad=$bg $(grep '^{' gpurun_out/attn23_$bg.jsonl | head -1 | cut -c1-200)"
done
DLLM_ATTN_BGRAD=shear timeout -k 10 300 python bench.py > gpurun_out/bench23_shear.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/bench23_shear.log; exit 1; }
echo "shear $(tail -1 gpurun_out/bench23_shear.log | cut -c1-200)"
