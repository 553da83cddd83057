#!/bin/bash
# Round 4: BART-large b=256 with the GELU forward GEMM persistent (DLLM_PP_PERSIST_GELU=1) vs one tile per workgroup
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4u
mkdir -p $O
for r in 1 2; do
  for v in 1 0; do
    DLLM_PP_PERSIST_GELU=$v timeout -k 10 300 python bench.py --model bart-large --batch-per-gpu 256 --steps 8 --warmup 3 > $O/bart_p${v}_${r}.log 2>&1 || { tail -5 $O/bart_p${v}_${r}.log; exit 1; }
    echo "persist_gelu=$v run $r: $(grep '"metric"' $O/bart_p${v}_${r}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
