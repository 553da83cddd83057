#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/ -q -m gpu -x > gpurun_out/gputests6.log 2>&1 || { echo GT_FAIL; grep -E "Error|assert|FAILED|passed|failed" gpurun_out/gputests6.log | tail -20; exit 1; }
tail -1 gpurun_out/gputests6.log
for b in 32 64; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --batch-per-gpu $b > gpurun_out/bench6_b$b.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/bench6_b$b.log; exit 1; }
  tail -1 gpurun_out/bench6_b$b.log
done
export VH_ROOT=$GRAFT_REPO_ROOT/gpurun_out/vh
timeout -k 10 300 python train-accelerator.py --model-ckpt t5-small --output-dir acc --synthetic 64 --batch-size 8 --max-source-length 256 --max-target-length 32 --gen-max-length 24 > gpurun_out/acc6.log 2>&1 || { echo ACC_FAIL; tail -20 gpurun_out/acc6.log; exit 1; }
grep rouge gpurun_out/acc6.log | tail -1
