#!/bin/bash
# Per-GPU batch sweep of the headline bench (t5-base 1024/128) on one box.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for b in 64 96 128 64; do
  timeout -k 10 300 python bench.py --batch-per-gpu $b > gpurun_out/b49_$b.log 2>&1 || { echo "B_FAIL $b"; tail -5 gpurun_out/b49_$b.log; continue; }
  echo "batch $b: $(tail -1 gpurun_out/b49_$b.log | cut -c90-190)"
done
python - <<'PY'
import torch
print("max mem GiB (last run not tracked)")
PY
