#!/bin/bash
# One-wave-per-SIMD GEMM main loop (csrc/gemm_pipe.h): numerics, A/B microbenches (fused 4 vs 5, wgrad 9 vs 11,
# plain GEMMs vs hipBLASLt).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "gemm or native_extension" --timeout 120 --timeout-method thread > gpurun_out/t37.log 2>&1 || { echo T_FAIL; grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/t37.log | tail -30; exit 1; }
tail -1 gpurun_out/t37.log
timeout -k 10 300 python -u tools/gemm_fused_bench.py > gpurun_out/gfb37.jsonl 2> gpurun_out/gfb37.err || { echo GFB_FAIL; tail -20 gpurun_out/gfb37.err; exit 1; }
cat gpurun_out/gfb37.jsonl
timeout -k 10 400 python -u tools/gemm_bench.py --no-torch > gpurun_out/gb37.jsonl 2> gpurun_out/gb37.err || { echo GB_FAIL; tail -20 gpurun_out/gb37.err; exit 1; }
cat gpurun_out/gb37.jsonl
timeout -k 10 400 python -u tools/gemm_plain_bench.py > gpurun_out/gpb37.jsonl 2> gpurun_out/gpb37.err || { echo GPB_FAIL; tail -20 gpurun_out/gpb37.err; exit 1; }
cat gpurun_out/gpb37.jsonl
