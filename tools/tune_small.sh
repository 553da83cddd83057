#!/bin/bash
# TunableOp tuning of GEMM shapes the shipped table lacks, merged into gpurun_out/tune_small/merged.csv, then the A/B of
# that table (DLLM_TUNABLEOP_TABLE) against the shipped one.
#   bash tools/tune_small.sh            # t5-base b=8 and b=1 (1024 / 128 decoder rows, 8192 / 1024 encoder rows)
#   TUNE_SET=bart bash tools/tune_small.sh   # bart-large 1024/1024 at b=1 and b=64 (the reference's train-torchrun shapes)
set -o pipefail
O=gpurun_out/tune_small
mkdir -p $O
if [ "${TUNE_SET:-t5}" = bart ]; then
  CFG_A="--model bart-large --src-len 1024 --tgt-len 1024 --batch-per-gpu 1"
  CFG_B="--model bart-large --src-len 1024 --tgt-len 1024 --batch-per-gpu 64"
  AB_A="$CFG_A --grad-accum 16 --steps 4 --warmup 2"
  AB_B="$CFG_B --steps 4 --warmup 2"
else
  CFG_A="--batch-per-gpu 8"
  CFG_B="--batch-per-gpu 1"
  AB_A="--batch-per-gpu 8 --grad-accum 16 --steps 6 --warmup 2"
  AB_B="--batch-per-gpu 1 --grad-accum 16 --steps 6 --warmup 2"
fi
TUNE_OUT=$O/a TUNE_TIMEOUT=500 bash tools/tunableop_tune.sh $CFG_A || exit 1
TUNE_OUT=$O/b TUNE_TIMEOUT=500 bash tools/tunableop_tune.sh $CFG_B || exit 1
python tools/merge_tunableop.py configs/tunableop/gfx950.csv $O/a/tunableop_results0.csv $O/b/tunableop_results0.csv \
  -o $O/merged.csv || exit 1
grep -c "" configs/tunableop/gfx950.csv $O/merged.csv
python tools/gpu_ab.py --tag tune_small_ab --reps 2 --env-arms "base=DLLM_TUNABLEOP=1,tuned=DLLM_TUNABLEOP_TABLE=$PWD/$O/merged.csv" \
  --bench "$AB_A" --bench "$AB_B"
