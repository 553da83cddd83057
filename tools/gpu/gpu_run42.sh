#!/bin/bash
# Ping-pong NT GEMM (variant 8) with branch-free steady-state k-tiles: numerics + A/B/A vs variant 4.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "gemm_fused" --timeout 120 --timeout-method thread > gpurun_out/t42.log 2>&1 || { echo T_FAIL; grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/t42.log | tail -30; exit 1; }
tail -1 gpurun_out/t42.log
timeout -k 10 400 python -u tools/gemm_plain_bench.py --variants 4,8,4,8 > gpurun_out/gp42.jsonl 2> gpurun_out/gp42.err || { echo GP_FAIL; tail -20 gpurun_out/gp42.err; exit 1; }
cat gpurun_out/gp42.jsonl
