#!/bin/bash
# End-to-end throughput of the three entry points at t5-base 1024/128 on one GPU (synthetic SAMSum-schema data,
# random init), next to bench.py; plus eval generation throughput.  gpurun -- bash tools/entry_bench.sh
set -o pipefail
mkdir -p gpurun_out/entry
O=gpurun_out/entry
common="--model-ckpt t5-base --synthetic 2560 --max-source-length 1024 --max-target-length 128 --output-dir /tmp/ebench"
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > $O/bench.log 2>&1 || exit 1
tail -1 $O/bench.log | cut -c1-160
timeout -k 10 900 python train-torchrun.py $common --batch-size 128 --grad-accum 1 --max-steps 12 \
  --evaluation-steps 1000000 --max-eval-samples 8 > $O/torchrun_b128.log 2>&1 || { tail -20 $O/torchrun_b128.log; exit 1; }
grep -h "train_runtime" $O/torchrun_b128.log | tail -1
timeout -k 10 900 python train-torchrun.py $common --batch-size 8 --grad-accum 16 --max-steps 5 \
  --evaluation-steps 1000000 --max-eval-samples 8 > $O/torchrun_b8_ga16.log 2>&1 || { tail -20 $O/torchrun_b8_ga16.log; exit 1; }
grep -h "train_runtime" $O/torchrun_b8_ga16.log | tail -1
timeout -k 10 900 python train-accelerator.py $common --batch-size 128 --max-steps 12 --max-eval-samples 8 \
  --gen-max-length 16 > $O/accelerator_b128.log 2>&1 || { tail -20 $O/accelerator_b128.log; exit 1; }
grep -h "train_samples_per_second" $O/accelerator_b128.log | tail -1
timeout -k 10 900 python tools/eval_bench.py --model t5-base --batch 64 --src-len 512 > $O/eval.log 2>&1 || { tail -20 $O/eval.log; exit 1; }
cat $O/eval.log | grep mode
timeout -k 10 900 python tools/loop_overhead.py --model t5-base --batch 128 --steps 10 > $O/loop.log 2>&1 || { tail -20 $O/loop.log; exit 1; }
tail -1 $O/loop.log
