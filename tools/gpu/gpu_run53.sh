#!/bin/bash
# After making the buffer-descriptor LDS-DMA opaque (no compiler vmcnt(0) before transposed reads): re-measure the
# ping-pong wgrad kernel (10 vs 9) and the fused GEMMs (8 vs 9: persistent d-relu / gelu).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/t53.log 2>&1 || { echo T_FAIL; grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/t53.log | tail -30; exit 1; }
tail -1 gpurun_out/t53.log
timeout -k 10 400 python -u tools/gemm_bench.py --no-torch --variants 9,10,9,10 > gpurun_out/gw53.jsonl 2> gpurun_out/gw53.err || { echo GW_FAIL; tail -20 gpurun_out/gw53.err; exit 1; }
cat gpurun_out/gw53.jsonl
timeout -k 10 300 python -u tools/gemm_fused_bench.py --variants 8,9,8,9 > gpurun_out/gf53.jsonl 2> gpurun_out/gf53.err || { echo GF_FAIL; tail -20 gpurun_out/gf53.err; exit 1; }
cat gpurun_out/gf53.jsonl
