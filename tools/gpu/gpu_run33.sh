#!/bin/bash
# norm_bwd with two rows per wave iteration: norm + model tests, bench, kernel stats.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -q -x -k "norm or native_extension or model or engine or fused_ffn" --timeout 180 --timeout-method thread > gpurun_out/t33.log 2>&1 || { echo T_FAIL; grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/t33.log | tail -30; exit 1; }
tail -1 gpurun_out/t33.log
timeout -k 10 300 python bench.py > gpurun_out/b33.log 2>&1 || { echo B_FAIL; tail -20 gpurun_out/b33.log; exit 1; }
tail -1 gpurun_out/b33.log
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof33 -o prof -- python $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof33.log 2>&1 || { echo PROF_FAIL; tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof33.log; exit 1; }
tail -1 $GRAFT_REPO_ROOT/gpurun_out/prof33.log
