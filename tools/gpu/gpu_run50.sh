#!/bin/bash
# Per-GPU batch sweep, larger batches.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for b in 128 160 192 256 128; do
  timeout -k 10 300 python bench.py --batch-per-gpu $b --steps 10 --warmup 3 > gpurun_out/b50_$b.log 2>&1 || { echo "B_FAIL $b"; grep -iE "memory|error" gpurun_out/b50_$b.log | tail -3; continue; }
  echo "batch $b: $(tail -1 gpurun_out/b50_$b.log | cut -c90-190)"
done
