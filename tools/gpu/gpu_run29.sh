#!/bin/bash
# Weight-gradient GEMM on 16x16x32 MFMA (csrc/gemm.hip variants 7-9): numerics, microbench vs the 32x32x16 variants.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "wgrad or native_extension" --timeout 120 --timeout-method thread > gpurun_out/t29.log 2>&1 || { echo T_FAIL; grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/t29.log | tail -30; exit 1; }
tail -1 gpurun_out/t29.log
timeout -k 10 400 python -u tools/gemm_bench.py --no-torch > gpurun_out/gb29.jsonl 2> gpurun_out/gb29.err || { echo GB_FAIL; tail -20 gpurun_out/gb29.err; exit 1; }
cat gpurun_out/gb29.jsonl
