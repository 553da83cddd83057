#!/bin/bash
# GEMM tuning at the b=64 shapes, then a 2-rank rehearsal of the multi-process bench on one GPU (gloo)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/tune9
DLLM_TUNABLEOP=tune DLLM_TUNABLEOP_DIR=gpurun_out/tune9 timeout -k 10 900 python bench.py --steps 2 --warmup 1 --batch-per-gpu 64 > gpurun_out/tune9.log 2>&1 || { echo TUNE_FAIL; tail -20 gpurun_out/tune9.log; exit 1; }
tail -1 gpurun_out/tune9.log | cut -c1-200
python tools/merge_tunableop.py gpurun_out/tune9/*.csv && cp configs/tunableop/gfx950.csv gpurun_out/gfx950_merged.csv
for b in 64 32; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --batch-per-gpu $b > gpurun_out/bench9_b$b.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/bench9_b$b.log; exit 1; }
  tail -1 gpurun_out/bench9_b$b.log | cut -c1-200
done
DLLM_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --batch-per-gpu 16 > gpurun_out/bench9_dp2.log 2>&1 || { echo DP2_FAIL; tail -30 gpurun_out/bench9_dp2.log; exit 1; }
grep '^{' gpurun_out/bench9_dp2.log | cut -c1-250
