#!/bin/bash
# Ping-pong NT GEMM tile-order groups (DLLM_GEMM_GRP): numerics + A/B in one process.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "gemm_fused or gemm_pp" --timeout 120 --timeout-method thread > gpurun_out/t43.log 2>&1 || { echo T_FAIL; grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/t43.log | tail -30; exit 1; }
tail -1 gpurun_out/t43.log
timeout -k 10 400 python -u tools/gemm_plain_bench.py --phases fwd --variants 8,8g2,8g4,8g8,8g16,8 > gpurun_out/gp43.jsonl 2> gpurun_out/gp43.err || { echo GP_FAIL; tail -20 gpurun_out/gp43.err; exit 1; }
cat gpurun_out/gp43.jsonl
