#!/bin/bash
# Per-GPU batch sweep of the bench default (t5-base 1024/128), interleaved on one box.
set -o pipefail
O=gpurun_out/batch
mkdir -p $O
for i in 1 2; do
  for b in 256 384 512; do
    timeout -k 10 400 python bench.py --steps 8 --warmup 3 --batch-per-gpu $b > $O/b${b}_$i.log 2>&1 || { tail -5 $O/b${b}_$i.log; exit 1; }
    echo "b=$b $(tail -1 $O/b${b}_$i.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], r["config"]["peak_mem_gb"])')"
  done
done
