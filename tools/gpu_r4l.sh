#!/bin/bash
# Round 4: w4 projection routing A/B (DLLM_W4_GEMM auto vs 0), t5-base b512 and bart-large b256, interleaved
set -o pipefail
O=gpurun_out/r4l
mkdir -p $O
for i in 1 2; do
  for m in auto 0; do
    DLLM_W4_GEMM=$m timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 > $O/t5_${m}_$i.log 2>&1 || { tail -20 $O/t5_${m}_$i.log; exit 1; }
    echo "t5 W4=$m: $(grep metric $O/t5_${m}_$i.log | cut -c100-200)"
  done
done
for i in 1 2; do
  for m in auto 0; do
    DLLM_W4_GEMM=$m timeout -k 10 600 python -u bench.py --model bart-large --batch-per-gpu 256 --steps 8 --warmup 3 > $O/bart_${m}_$i.log 2>&1 || { tail -20 $O/bart_${m}_$i.log; exit 1; }
    echo "bart W4=$m: $(grep metric $O/bart_${m}_$i.log | cut -c100-200)"
  done
done
