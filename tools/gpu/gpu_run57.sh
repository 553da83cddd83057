#!/bin/bash
# Context-parallel ring attention: native block numerics (W virtual ranks on one GPU) and the W=1 op.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -v -x -k "context_parallel or ring_attention" --timeout 120 --timeout-method thread > gpurun_out/t57.log 2>&1 || { echo T_FAIL; grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/t57.log | tail -30; exit 1; }
tail -3 gpurun_out/t57.log
