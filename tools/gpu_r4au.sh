#!/bin/bash
# Round 4: gated-GELU FFN on the fused GEMMs for wider models too (DLLM_GATED_MAX_D=4096) vs the default (d <= 768),
# now that the gated backward epilogue is staged: flan-t5-large b=32, flan-t5-xl b=16, alternating
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4au
mkdir -p $O
for r in 1 2; do
  for md in 4096 768; do
    for m in "flan-t5-large 32" "flan-t5-xl 16"; do
      set -- $m
      DLLM_GATED_MAX_D=$md timeout -k 10 300 python bench.py --model $1 --batch-per-gpu $2 --steps 8 --warmup 3 > $O/${1}_${md}_${r}.log 2>&1 || { tail -5 $O/${1}_${md}_${r}.log; exit 1; }
      echo "$1 b$2 maxd=$md $r: $(grep '"metric"' $O/${1}_${md}_${r}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
    done
  done
done
