#!/bin/bash
# Whole-step A/B on one box: fused FFN GEMM variant 4 vs 8 (ping-pong), alternating.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 4 8 4 8; do
  DLLM_GEMM_FUSED_VARIANT=$v timeout -k 10 300 python bench.py > gpurun_out/b45_$v.log 2>&1 || { echo B_FAIL; tail -20 gpurun_out/b45_$v.log; exit 1; }
  echo "variant $v: $(tail -1 gpurun_out/b45_$v.log | cut -c1-200)"
done
