#!/bin/bash
# wgrad GEMM kernel: numerics first (stop on any failure), then microbenchmark vs hipBLASLt
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -k "gemm_wgrad or wgrad_path" > gpurun_out/gemm11_tests.log 2>&1 || { echo GT_FAIL; grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/gemm11_tests.log | tail -20; exit 1; }
tail -1 gpurun_out/gemm11_tests.log
timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/gemm11_bench.jsonl 2>&1 || { echo GB_FAIL; tail -20 gpurun_out/gemm11_bench.jsonl; exit 1; }
cat gpurun_out/gemm11_bench.jsonl
