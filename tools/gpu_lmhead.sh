#!/bin/bash
# LM head at the b=512 default: vocabulary-chunked CE (default above 2 GiB of logits) vs the full-logits path.
set -o pipefail
O=gpurun_out/lmhead
mkdir -p $O
for i in 1 2; do
  for mb in 2048 -1; do
    DLLM_LMHEAD_FULL_MB=$mb timeout -k 10 400 python bench.py --steps 8 --warmup 3 > $O/m${mb}_$i.log 2>&1 || { tail -5 $O/m${mb}_$i.log; exit 1; }
    echo "full_mb=$mb $(tail -1 $O/m${mb}_$i.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], r["config"]["peak_mem_gb"])')"
  done
done
