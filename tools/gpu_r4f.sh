#!/bin/bash
# Round 4: side-stream crossover (batch 16 / 32 / 64 / 128, forced on vs off) + the reference-loop entry point at b1
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4f
mkdir -p $O
for b in 16 32 64 128; do
  for s in 1 0; do
    DLLM_WGRAD_STREAM=$s timeout -k 10 600 python -u bench.py --batch-per-gpu $b --steps 8 --warmup 3 > $O/b${b}_s$s.log 2>&1 || { tail -20 $O/b${b}_s$s.log; exit 1; }
    echo "b$b stream=$s: $(grep metric $O/b${b}_s$s.log | cut -c100-200)"
  done
done
common="--model-ckpt t5-base --synthetic 2560 --max-source-length 1024 --max-target-length 128 --output-dir /tmp/ebench"
timeout -k 10 600 python -u train-accelerator.py $common --batch-size 1 --max-steps 120 --max-eval-samples 4 \
  --gen-max-length 8 > $O/acc_b1.log 2>&1 || { tail -20 $O/acc_b1.log; exit 1; }
echo "accelerator b1 (auto): $(grep -h train_samples_per_second $O/acc_b1.log | tail -1)"
