#!/bin/bash
# Other BASELINE.json configs on 1 GPU: this framework vs the HF stack (same synthetic shapes)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/cfg17
step() {  # name, timeout, cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > gpurun_out/cfg17/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep '^{' gpurun_out/cfg17/$name.log | tail -1 | cut -c1-260)"
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "STOP after $name"; exit 1; fi
  [ $rc -ne 0 ] && tail -3 gpurun_out/cfg17/$name.log
  return 0
}
step ours_bart_large_b32 420 python bench.py --model bart-large --batch-per-gpu 32 --steps 8 --warmup 3
step ours_t5_large_b32 420 python bench.py --model t5-large --batch-per-gpu 32 --steps 8 --warmup 3
step ours_flan_t5_xl_b16 600 python bench.py --model flan-t5-xl --batch-per-gpu 16 --steps 5 --warmup 2
step hf_bart_large_b32 420 python tools/hf_comparator.py --model bart-large --batch 32 --steps 5 --warmup 2
step hf_t5_large_b16 420 python tools/hf_comparator.py --model t5-large --batch 16 --steps 5 --warmup 2
step hf_flan_t5_xl_b8 600 python tools/hf_comparator.py --model flan-t5-xl --batch 8 --steps 4 --warmup 2
