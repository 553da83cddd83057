#!/bin/bash
# The reference's default training step (bart-large-cnn, 1024 source / 1024 target, batch 1 x GA 16 through
# train-torchrun.py: ref/valohai.yaml:10, ref/train-torchrun.py:99,102,119,126) in the round-start tree (GATE_BASE) and the
# current tree, interleaved, REPS rounds; steady samples/s per run in gpurun_out/<tag>/entry.txt.
set -o pipefail
TAG=${1:-entry_bart}
REPS=${2:-2}
BASE=${GATE_BASE:-ab/r6base}
O=gpurun_out/$TAG
mkdir -p $O
cmd="train-torchrun.py --model-ckpt bart-large-cnn --synthetic 2048 --max-source-length 1024 --max-target-length 1024 \
--output-dir /tmp/ebg --batch-size 1 --grad-accum 16 --max-steps 16 --evaluation-steps 1000000 --max-eval-samples 8"
for rep in $(seq 1 $REPS); do
  for arm in base cur; do
    dir=.; [ $arm = base ] && dir=$BASE
    log=$O/bart_${arm}_${rep}.log
    (cd $dir && timeout -k 10 600 python $cmd) > $log 2>&1 || { echo "FAILED $arm"; tail -20 $log; exit 1; }
    v=$(grep -ho '"train_steady_samples_per_second": [0-9.]*' $log | tail -1 | awk '{print $2}')
    echo "bart_cnn_b1_ga16 $arm rep$rep steady_samples_per_s $v" | tee -a $O/entry.txt
  done
done
