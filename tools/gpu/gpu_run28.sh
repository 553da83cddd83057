#!/bin/bash
# Fused-epilogue FFN GEMM (csrc/gemm_fused.hip): numerics vs fp32 torch, microbench vs hipBLASLt + activation
# kernels, whole-model fused vs unfused, then the headline bench with the FFN fusion off / on.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "gemm_fused or native_extension" --timeout 120 --timeout-method thread > gpurun_out/t28.log 2>&1 || { echo T_FAIL; grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/t28.log | tail -30; exit 1; }
tail -1 gpurun_out/t28.log
timeout -k 10 300 python -u tools/gemm_fused_bench.py > gpurun_out/gfb28.jsonl 2> gpurun_out/gfb28.err || { echo GFB_FAIL; tail -20 gpurun_out/gfb28.err; exit 1; }
cat gpurun_out/gfb28.jsonl
timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py -q -x --timeout 180 --timeout-method thread > gpurun_out/m28.log 2>&1 || { echo M_FAIL; grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/m28.log | tail -30; exit 1; }
tail -1 gpurun_out/m28.log
DLLM_FUSED_FFN=0 timeout -k 10 300 python bench.py > gpurun_out/b28_off.log 2>&1 || { echo B0_FAIL; tail -20 gpurun_out/b28_off.log; exit 1; }
tail -1 gpurun_out/b28_off.log
timeout -k 10 300 python bench.py > gpurun_out/b28_on.log 2>&1 || { echo B1_FAIL; tail -20 gpurun_out/b28_on.log; exit 1; }
tail -1 gpurun_out/b28_on.log
DLLM_ATTN_MASK_STREAM=1 timeout -k 10 300 python bench.py > gpurun_out/b28_ms.log 2>&1 || { echo B2_FAIL; tail -20 gpurun_out/b28_ms.log; exit 1; }
tail -1 gpurun_out/b28_ms.log
