#!/bin/bash
# Round 4: wgrad split-count A/B (tail-filling vs legacy fill-once), t5-base b512 bench, interleaved
set -o pipefail
O=gpurun_out/r4j
mkdir -p $O
for i in 1 2; do
  for m in new legacy; do
    if [ $m = legacy ]; then export DLLM_WGRAD_SPLIT_LEGACY=1; else unset DLLM_WGRAD_SPLIT_LEGACY; fi
    timeout -k 10 600 python -u bench.py --steps 12 --warmup 3 > $O/${m}_$i.log 2>&1 || { tail -20 $O/${m}_$i.log; exit 1; }
    echo "$m: $(grep metric $O/${m}_$i.log | cut -c1-200)"
  done
done
