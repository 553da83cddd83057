#!/bin/bash
# TunableOp tuning of the micro-batch GEMM shapes (t5-base b=8 and b=1: 1024 / 128 decoder rows, 8192 / 1024 encoder
# rows) that the shipped table lacks, merged into gpurun_out/tune_small/merged.csv; then the A/B of that table
# (DLLM_TUNABLEOP_TABLE) against the shipped one at b=8 x GA16 and b=1 x GA16.
set -o pipefail
O=gpurun_out/tune_small
mkdir -p $O
TUNE_OUT=$O/b8 TUNE_TIMEOUT=500 bash tools/tunableop_tune.sh --batch-per-gpu 8 || exit 1
TUNE_OUT=$O/b1 TUNE_TIMEOUT=400 bash tools/tunableop_tune.sh --batch-per-gpu 1 || exit 1
python tools/merge_tunableop.py configs/tunableop/gfx950.csv $O/b8/tunableop_results0.csv $O/b1/tunableop_results0.csv \
  -o $O/merged.csv || exit 1
grep -c "" configs/tunableop/gfx950.csv $O/merged.csv
python tools/gpu_ab.py --tag tune_small_ab --reps 2 --env-arms "base=DLLM_TUNABLEOP=1,tuned=DLLM_TUNABLEOP_TABLE=$PWD/$O/merged.csv" \
  --bench "--batch-per-gpu 8 --grad-accum 16 --steps 6 --warmup 2" --bench "--batch-per-gpu 1 --grad-accum 16 --steps 6 --warmup 2"
