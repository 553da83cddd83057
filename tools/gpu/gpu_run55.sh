#!/bin/bash
# TunableOp pass for the batch-128 GEMM shapes (enc 131072 / dec 16384 tokens) missing from the in-tree table.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/tune55
DLLM_TUNABLEOP=tune DLLM_TUNABLEOP_DIR=$GRAFT_REPO_ROOT/gpurun_out/tune55 PYTORCH_TUNABLEOP_VERBOSE=1 \
  timeout -k 10 1000 python bench.py --steps 1 --warmup 1 > gpurun_out/tune55/log.txt 2>&1 || { echo TUNE_FAIL; tail -20 gpurun_out/tune55/log.txt; exit 1; }
tail -1 gpurun_out/tune55/log.txt
ls -la gpurun_out/tune55
