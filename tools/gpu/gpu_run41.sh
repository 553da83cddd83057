#!/bin/bash
# Deep-ring BK32 (variants 5-7) and ping-pong (variant 8) fused GEMMs: numerics, then plain + fused microbench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "gemm_fused" --timeout 120 --timeout-method thread > gpurun_out/t41.log 2>&1 || { echo T_FAIL; grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/t41.log | tail -30; exit 1; }
tail -1 gpurun_out/t41.log
timeout -k 10 400 python -u tools/gemm_plain_bench.py --variants 4,5,7,8 > gpurun_out/gp41.jsonl 2> gpurun_out/gp41.err || { echo GP_FAIL; tail -20 gpurun_out/gp41.err; exit 1; }
cat gpurun_out/gp41.jsonl
timeout -k 10 300 python -u tools/gemm_fused_bench.py --variants 4,5,7,8 > gpurun_out/gf41.jsonl 2> gpurun_out/gf41.err || { echo GF_FAIL; tail -20 gpurun_out/gf41.err; exit 1; }
cat gpurun_out/gf41.jsonl
