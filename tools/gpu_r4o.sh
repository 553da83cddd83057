#!/bin/bash
# Round 4: BART-large FFN fused (GELU epilogue GEMMs) vs unfused (hipBLASLt + activation kernels), b256, interleaved
set -o pipefail
O=gpurun_out/r4o
mkdir -p $O
for i in 1 2; do
  for m in 1 0; do
    DLLM_FUSED_FFN=$m timeout -k 10 600 python -u bench.py --model bart-large --batch-per-gpu 256 --steps 8 --warmup 3 > $O/bart_ffn${m}_$i.log 2>&1 || { tail -20 $O/bart_ffn${m}_$i.log; exit 1; }
    echo "bart fused_ffn=$m: $(grep metric $O/bart_ffn${m}_$i.log | cut -c150-260)"
  done
done
