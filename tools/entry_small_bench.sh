#!/bin/bash
# The reference's own micro-batches through the entry points (t5-base 1024/128, one GPU, synthetic data): train-torchrun
# at batch 1 x GA 16 (ref/train-torchrun.py:119,126; accumulation passes coalesced when HBM allows) and batch 8 x GA 16,
# train-accelerator at batch 1 (one AdamW step per sample).  gpurun -- bash tools/entry_small_bench.sh
set -o pipefail
mkdir -p gpurun_out/entry_small
O=gpurun_out/entry_small
common="--model-ckpt t5-base --synthetic 4096 --max-source-length 1024 --max-target-length 128 --output-dir /tmp/esb"
run() {
  name=$1; shift
  timeout -k 10 600 python "$@" > $O/$name.log 2>&1 || { tail -20 $O/$name.log; exit 1; }
  grep -h "train_runtime\|train_samples_per_second" $O/$name.log | tail -1 | cut -c1-400
}
run torchrun_b1_ga16 train-torchrun.py $common --batch-size 1 --grad-accum 16 --max-steps 24 \
  --evaluation-steps 1000000 --max-eval-samples 8
run torchrun_b8_ga16 train-torchrun.py $common --batch-size 8 --grad-accum 16 --max-steps 16 \
  --evaluation-steps 1000000 --max-eval-samples 8
run accelerator_b1 train-accelerator.py $common --batch-size 1 --max-steps 200 --max-eval-samples 8 --gen-max-length 16
# the reference's default training step itself: bart-large-cnn, 1024 source / 1024 target, batch 1 x GA 16
# (ref/valohai.yaml:10, ref/train-torchrun.py:99,102,119,126)
bart="--model-ckpt bart-large-cnn --synthetic 2048 --max-source-length 1024 --max-target-length 1024 --output-dir /tmp/esb2"
run torchrun_bart_cnn_b1_ga16 train-torchrun.py $bart --batch-size 1 --grad-accum 16 --max-steps 16 \
  --evaluation-steps 1000000 --max-eval-samples 8
