#!/bin/bash
# BART-large (bias- and dropout-free attention): dK/dV at 3 WG/CU (NB=2 ring, default) vs 2 WG/CU (NB=3 ring with the
# prefetched MFMA operands), and T5 with the cross-attention dK/dV the same way; interleaved on one box.
set -o pipefail
O=gpurun_out/bartocc
mkdir -p $O
for i in 1 2; do
  for occ in 3 2; do
    DLLM_ATTN_DKDV_OCC=$occ timeout -k 10 400 python bench.py --model bart-large --batch-per-gpu 256 --steps 5 --warmup 2 > $O/bart_$occ_$i.log 2>&1 || { tail -5 $O/bart_$occ_$i.log; exit 1; }
    echo "bart occ=$occ $(tail -1 $O/bart_$occ_$i.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')"
  done
  for v in 1 0; do
    DLLM_ATTN_DKDV_OCC_DR=$v timeout -k 10 400 python bench.py --steps 8 --warmup 3 > $O/t5_$v_$i.log 2>&1 || { tail -5 $O/t5_$v_$i.log; exit 1; }
    echo "t5 occ_dr=$v $(tail -1 $O/t5_$v_$i.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')"
  done
done
