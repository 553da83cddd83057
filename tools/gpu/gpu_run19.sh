#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/cfg19
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > gpurun_out/cfg19/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep '^{' gpurun_out/cfg19/$name.log | tail -1 | cut -c1-300)"
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "STOP after $name"; exit 1; fi
  [ $rc -ne 0 ] && tail -3 gpurun_out/cfg19/$name.log
  return 0
}
timeout -k 10 600 python -m pytest tests/ -q -m gpu -x > gpurun_out/gputests19.log 2>&1 || { echo GT_FAIL; grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/gputests19.log | tail -20; exit 1; }
tail -1 gpurun_out/gputests19.log
step bart_large_b32 420 python bench.py --model bart-large --batch-per-gpu 32 --steps 8 --warmup 3
step t5base_b64_ckpt 420 python bench.py --grad-ckpt --steps 8 --warmup 3
step flan_xl_long_s4096_b8_ckpt 900 python bench.py --model flan-t5-xl --src-len 4096 --tgt-len 256 --batch-per-gpu 8 --grad-ckpt --steps 4 --warmup 2
