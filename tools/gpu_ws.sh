#!/bin/bash
# hipBLASLt workspace: torch default vs 256 MiB (HIPBLASLT_WORKSPACE_SIZE in KiB), t5-base b=512 and bart-large b=256.
set -o pipefail
O=gpurun_out/ws
mkdir -p $O
for i in 1 2; do
  for ws in default 262144; do
    if [ $ws = default ]; then unset HIPBLASLT_WORKSPACE_SIZE; else export HIPBLASLT_WORKSPACE_SIZE=$ws; fi
    timeout -k 10 400 python bench.py --steps 8 --warmup 3 > $O/t5_${ws}_$i.log 2>&1 || { tail -5 $O/t5_${ws}_$i.log; exit 1; }
    echo "t5 ws=$ws $(tail -1 $O/t5_${ws}_$i.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')"
    timeout -k 10 400 python bench.py --model bart-large --steps 5 --warmup 2 > $O/bart_${ws}_$i.log 2>&1 || { tail -5 $O/bart_${ws}_$i.log; exit 1; }
    echo "bart ws=$ws $(tail -1 $O/bart_${ws}_$i.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')"
  done
done
