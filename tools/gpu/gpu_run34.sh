#!/bin/bash
# GEMM fragment preload variants (fused 4 vs 3, wgrad 10 vs 9): numerics, A/B microbenches in one process each.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "gemm or native_extension" --timeout 120 --timeout-method thread > gpurun_out/t34.log 2>&1 || { echo T_FAIL; grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/t34.log | tail -30; exit 1; }
tail -1 gpurun_out/t34.log
timeout -k 10 300 python -u tools/gemm_fused_bench.py > gpurun_out/gfb34.jsonl 2> gpurun_out/gfb34.err || { echo GFB_FAIL; tail -20 gpurun_out/gfb34.err; exit 1; }
cat gpurun_out/gfb34.jsonl
timeout -k 10 400 python -u tools/gemm_bench.py --no-torch > gpurun_out/gb34.jsonl 2> gpurun_out/gb34.err || { echo GB_FAIL; tail -20 gpurun_out/gb34.err; exit 1; }
cat gpurun_out/gb34.jsonl
