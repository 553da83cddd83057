#!/bin/bash
# Round 4: bench lines for the new BART-family model types (1024/128 tokens where the model allows, bf16)
set -o pipefail
O=gpurun_out/r4m
mkdir -p $O
for c in "mbart:--model mbart-large-cc25 --batch-per-gpu 128" "pegasus:--model pegasus-large --batch-per-gpu 128" "marian:--model opus-mt-en-de --batch-per-gpu 256 --src-len 512" "nllb:--model nllb-200-distilled-600m --batch-per-gpu 128"; do
  tag=${c%%:*}; args=${c#*:}
  timeout -k 10 600 python -u bench.py $args --steps 6 --warmup 3 > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }
  echo "$tag: $(grep metric $O/$tag.log | cut -c80-330)"
done
