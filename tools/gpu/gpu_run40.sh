#!/bin/bash
# dK/dV query tiles by LDS-DMA two tiles ahead (3-deep ring), padded lse/delta rows: attention tests + microbench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "attention or native_extension" --timeout 120 --timeout-method thread > gpurun_out/t40.log 2>&1 || { echo T_FAIL; grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/t40.log | tail -30; exit 1; }
tail -1 gpurun_out/t40.log
timeout -k 10 400 python -u tools/attn_bench.py > gpurun_out/ab40.jsonl 2> gpurun_out/ab40.err || { echo AB_FAIL; tail -20 gpurun_out/ab40.err; exit 1; }
cat gpurun_out/ab40.jsonl
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py -q -x --timeout 180 --timeout-method thread > gpurun_out/m40.log 2>&1 || { echo M_FAIL; grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/m40.log | tail -30; exit 1; }
tail -1 gpurun_out/m40.log
timeout -k 10 300 python bench.py > gpurun_out/b40.log 2>&1 || { echo B_FAIL; tail -20 gpurun_out/b40.log; exit 1; }
tail -1 gpurun_out/b40.log
