#!/bin/bash
# Round 4: small-batch dQ occupancy A/B (3 per CU where it saves a round vs always 2), t5-base b8 x GA16, interleaved
set -o pipefail
O=gpurun_out/r4n
mkdir -p $O
for i in 1 2; do
  for m in auto 2; do
    if [ $m = 2 ]; then export DLLM_ATTN_DQ_OCC=2; else unset DLLM_ATTN_DQ_OCC; fi
    timeout -k 10 600 python -u bench.py --batch-per-gpu 8 --grad-accum 16 --steps 8 --warmup 3 > $O/b8_${m}_$i.log 2>&1 || { tail -20 $O/b8_${m}_$i.log; exit 1; }
    echo "b8xGA16 dq_occ=$m: $(grep metric $O/b8_${m}_$i.log | cut -c100-200)"
  done
done
