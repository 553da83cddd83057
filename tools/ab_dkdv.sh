#!/bin/bash
# A/B bench on one box: alternate env settings
set -o pipefail
mkdir -p gpurun_out/ab
for i in 1 2; do
  DLLM_ATTN_DKDV=1 timeout -k 10 300 python bench.py --steps 15 --warmup 3 > gpurun_out/ab/v1_$i.log 2>&1 || exit 1
  echo "v1 $(tail -1 gpurun_out/ab/v1_$i.log | cut -c1-120)"
  timeout -k 10 300 python bench.py --steps 15 --warmup 3 > gpurun_out/ab/v2_$i.log 2>&1 || exit 1
  echo "v2 $(tail -1 gpurun_out/ab/v2_$i.log | cut -c1-120)"
done
