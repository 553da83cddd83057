#!/bin/bash
# Default fused GEMM variant 9 (persistent for store-only epilogues): tests + whole-step A/B vs variant 8.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/t47.log 2>&1 || { echo T_FAIL; grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/t47.log | tail -30; exit 1; }
tail -1 gpurun_out/t47.log
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py -q -x --timeout 180 --timeout-method thread > gpurun_out/m47.log 2>&1 || { echo M_FAIL; grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/m47.log | tail -30; exit 1; }
tail -1 gpurun_out/m47.log
for v in 8 9 8 9; do
  DLLM_GEMM_FUSED_VARIANT=$v timeout -k 10 300 python bench.py > gpurun_out/b47_$v.log 2>&1 || { echo B_FAIL; tail -20 gpurun_out/b47_$v.log; exit 1; }
  echo "variant $v: $(tail -1 gpurun_out/b47_$v.log | cut -c100-200)"
done
