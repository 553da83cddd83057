#!/bin/bash
# No-regression gate across BASELINE.json's configs: every config below, interleaved between the
# round-start tree (arm "base": a checkout of the round's first commit with its own library, built under ab/) and the
# current tree (arm "cur"), REPS rounds, medians per arm and the delta in gpurun_out/<tag>/bench_table.txt.
# A config more than 1 % below base is a finding to fix.
#
#   git worktree add ab/r4base <round-start commit> && (cd ab/r4base && python tools/build_native.py)
#   gpurun --timeout 1200 -- bash tools/regression_gate.sh gate [REPS]
set -o pipefail
TAG=${1:-gate}
REPS=${2:-2}
BASE=${GATE_BASE:-ab/r4base}
exec_args=(
  --tag "$TAG" --tree-arms "base=$BASE,cur=." --reps "$REPS" --bench-limit 480
  --bench "--steps 10 --warmup 3"
  --bench "--model bart-large --batch-per-gpu 256 --steps 6 --warmup 2"
  --bench "--model t5-large --batch-per-gpu 32 --steps 6 --warmup 2"
  --bench "--model flan-t5-xl --batch-per-gpu 16 --steps 5 --warmup 2"
  --bench "--dtype fp32 --batch-per-gpu 16 --steps 6 --warmup 2"
)
# GATE_SMALL=1: also the reference's small micro-batch / long-target shapes (train-torchrun: batch 1 x GA 16, BART
# 1024 / 1024)
# GATE_SMALL=only: the small shapes alone (the two halves fit one gpurun call each)
if [ "${GATE_SMALL:-0}" = only ]; then
  exec_args=(--tag "$TAG" --tree-arms "base=$BASE,cur=." --reps "$REPS" --bench-limit 480)
fi
if [ "${GATE_SMALL:-0}" != 0 ]; then
  exec_args+=(
    --bench "--model bart-large --src-len 1024 --tgt-len 1024 --batch-per-gpu 64 --steps 5 --warmup 2"
    --bench "--batch-per-gpu 8 --grad-accum 16 --steps 6 --warmup 2"
    --bench "--batch-per-gpu 1 --grad-accum 16 --steps 6 --warmup 2"
  )
fi
python tools/gpu_ab.py "${exec_args[@]}"
