#!/bin/bash
# Persistent ping-pong GEMM (variant 9): numerics, then A/B/A/B vs variant 8 (plain fwd/dgrad + fused FFN).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/t46.log 2>&1 || { echo T_FAIL; grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/t46.log | tail -30; exit 1; }
tail -1 gpurun_out/t46.log
timeout -k 10 400 python -u tools/gemm_plain_bench.py --variants 8,9,8,9 > gpurun_out/gp46.jsonl 2> gpurun_out/gp46.err || { echo GP_FAIL; tail -20 gpurun_out/gp46.err; exit 1; }
cat gpurun_out/gp46.jsonl
timeout -k 10 300 python -u tools/gemm_fused_bench.py --variants 8,9,8,9 > gpurun_out/gf46.jsonl 2> gpurun_out/gf46.err || { echo GF_FAIL; tail -20 gpurun_out/gf46.err; exit 1; }
cat gpurun_out/gf46.jsonl
