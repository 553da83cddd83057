#!/bin/bash
# Chunked long-sequence attention: numerics at 8K / 16K, then t5-base training steps at 16K / 32K encoder tokens on one GPU.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -v -x -k "chunked or context_parallel or ring_attention" --timeout 200 --timeout-method thread > gpurun_out/t59.log 2>&1 || { echo T_FAIL; grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/t59.log | tail -30; exit 1; }
tail -2 gpurun_out/t59.log
for S in 16384 32768; do
  timeout -k 10 400 python bench.py --batch-per-gpu 1 --src-len $S --steps 5 --warmup 2 > gpurun_out/b59_$S.log 2>&1 || { echo B_FAIL; tail -20 gpurun_out/b59_$S.log; exit 1; }
  tail -1 gpurun_out/b59_$S.log
done
timeout -k 10 400 python bench.py --model flan-t5-xl --batch-per-gpu 1 --src-len 16384 --grad-ckpt --steps 3 --warmup 1 > gpurun_out/b59_xl.log 2>&1 || { echo BXL_FAIL; tail -20 gpurun_out/b59_xl.log; exit 1; }
tail -1 gpurun_out/b59_xl.log
