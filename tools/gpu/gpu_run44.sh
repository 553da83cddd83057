#!/bin/bash
# Ping-pong GEMM for k-major B (dgrad) + default switch: numerics, A/B vs variant 4, model tests, bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/t44.log 2>&1 || { echo T_FAIL; grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/t44.log | tail -30; exit 1; }
tail -1 gpurun_out/t44.log
timeout -k 10 300 python -u tools/gemm_fused_bench.py --variants 4,8,4,8 > gpurun_out/gf44.jsonl 2> gpurun_out/gf44.err || { echo GF_FAIL; tail -20 gpurun_out/gf44.err; exit 1; }
cat gpurun_out/gf44.jsonl
timeout -k 10 400 python -u tools/gemm_plain_bench.py --phases dgrad --variants 4,8,4,8 > gpurun_out/gp44.jsonl 2> gpurun_out/gp44.err || { echo GP_FAIL; tail -20 gpurun_out/gp44.err; exit 1; }
cat gpurun_out/gp44.jsonl
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py -q -x --timeout 180 --timeout-method thread > gpurun_out/m44.log 2>&1 || { echo M_FAIL; grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/m44.log | tail -30; exit 1; }
tail -1 gpurun_out/m44.log
timeout -k 10 300 python bench.py > gpurun_out/b44.log 2>&1 || { echo B_FAIL; tail -20 gpurun_out/b44.log; exit 1; }
tail -1 gpurun_out/b44.log
