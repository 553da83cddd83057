#!/bin/bash
# Ping-pong wgrad kernel (variant 10): numerics + A/B/A/B vs variant 9.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "wgrad" --timeout 120 --timeout-method thread > gpurun_out/t48.log 2>&1 || { echo T_FAIL; grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/t48.log | tail -30; exit 1; }
tail -1 gpurun_out/t48.log
timeout -k 10 400 python -u tools/gemm_bench.py --no-torch --variants 9,10,9,10 > gpurun_out/gw48.jsonl 2> gpurun_out/gw48.err || { echo GW_FAIL; tail -20 gpurun_out/gw48.err; exit 1; }
cat gpurun_out/gw48.jsonl
