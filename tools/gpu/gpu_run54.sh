#!/bin/bash
# ReLU derivative bit mask (fwd writes bits, bwd stages them by LDS-DMA, persistent d-relu): tests + whole-step A/B.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/t54.log 2>&1 || { echo T_FAIL; grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/t54.log | tail -30; exit 1; }
tail -1 gpurun_out/t54.log
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py -q -x --timeout 180 --timeout-method thread > gpurun_out/m54.log 2>&1 || { echo M_FAIL; grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/m54.log | tail -30; exit 1; }
tail -1 gpurun_out/m54.log
for m in 0 1 0 1; do
  DLLM_RELU_MASK=$m timeout -k 10 300 python bench.py > gpurun_out/b54_$m.log 2>&1 || { echo B_FAIL; tail -20 gpurun_out/b54_$m.log; exit 1; }
  echo "mask $m: $(tail -1 gpurun_out/b54_$m.log | cut -c90-190)"
done
