#!/bin/bash
# Two ranks on ONE GPU over gloo (RCCL refuses two ranks per device): exercises the multi-rank path of bench.py
# (broadcast, bucketed overlapped reducer with the ready-order rebuild, fp32 gradients) with the real kernels.
set -o pipefail
mkdir -p gpurun_out/gloo2
export DLLM_DIST_BACKEND=gloo
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29611 bench.py --gpus 2 --steps 4 --warmup 2 --batch-per-gpu 16 > gpurun_out/gloo2/bench.log 2>&1 \
  || { tail -30 gpurun_out/gloo2/bench.log; exit 1; }
tail -1 gpurun_out/gloo2/bench.log | cut -c1-400
# gradient accumulation (deferred weight gradients inside the captured window, overlap schedule on the last pass)
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29613 bench.py --gpus 2 --steps 3 --warmup 2 --batch-per-gpu 8 --grad-accum 2 > gpurun_out/gloo2/bench_ga.log 2>&1 \
  || { tail -30 gpurun_out/gloo2/bench_ga.log; exit 1; }
tail -1 gpurun_out/gloo2/bench_ga.log | cut -c1-400
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29612 train-torchrun.py --model-ckpt t5-small --synthetic 256 --batch-size 8 --grad-accum 2 \
  --max-steps 6 --evaluation-steps 3 --max-eval-samples 8 --output-dir /tmp/g2 > gpurun_out/gloo2/torchrun.log 2>&1 \
  || { tail -30 gpurun_out/gloo2/torchrun.log; exit 1; }
grep -h "train_runtime\|eval_loss" gpurun_out/gloo2/torchrun.log | tail -3
