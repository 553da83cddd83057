#!/bin/bash
# TunableOp re-tune at the micro-batch shapes of the reference loops (b=1 and b=8 token rows, GA windows): three
# tools/tunableop_tune.sh runs, results in gpurun_out/tune_<cfg>/ (merge with tools/merge_tunableop.py).
set -o pipefail
export TMPDIR=/tmp
for cfg in "b1ga16:--batch-per-gpu 1 --grad-accum 16" "b1:--batch-per-gpu 1" "b8ga16:--batch-per-gpu 8 --grad-accum 16"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  TUNE_OUT=gpurun_out/tune_$tag TUNE_TIMEOUT=500 timeout -k 10 560 bash tools/tunableop_tune.sh $args || exit 1
  echo "tuned $tag"
done
