#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x > gpurun_out/kt3.log 2>&1 || { echo KT_FAIL; grep -E "Error|assert|FAILED|passed|failed" gpurun_out/kt3.log | tail -20; exit 1; }
tail -1 gpurun_out/kt3.log
for b in 32 64; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --batch-per-gpu $b > gpurun_out/bench3_b$b.log 2>&1 || { echo BENCH_FAIL $b; tail -30 gpurun_out/bench3_b$b.log; exit 1; }
  tail -1 gpurun_out/bench3_b$b.log
done
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof3 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --batch-per-gpu 32 > $GRAFT_REPO_ROOT/gpurun_out/prof3.log 2>&1 || { echo PROF_FAIL; tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof3.log; exit 1; }
echo PROF_OK
