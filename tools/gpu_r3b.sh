#!/bin/bash
# Round-3 measurements: small-batch (reference micro-batches) graph vs eager, fp32 training, entry point in fp32,

set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3b
mkdir -p $O
run() {  # tag, timeout, command...
  local tag=$1 to=$2; shift 2
  echo "[r3b] $tag"
  timeout -k 10 $to "$@" > $O/$tag.log 2>&1 || { echo "[r3b] $tag failed rc=$?"; tail -15 $O/$tag.log; exit 1; }
  grep -h '"metric"' $O/$tag.log | tail -1 | cut -c1-420
}
run b8ga16_graph 400 python -u bench.py --batch-per-gpu 8 --grad-accum 16 --steps 5 --warmup 2 --graph on
run b8ga16_eager 400 python -u bench.py --batch-per-gpu 8 --grad-accum 16 --steps 5 --warmup 2 --graph off
run b1ga16_graph 400 python -u bench.py --batch-per-gpu 1 --grad-accum 16 --steps 5 --warmup 2 --graph on
run b1ga16_eager 400 python -u bench.py --batch-per-gpu 1 --grad-accum 16 --steps 5 --warmup 2 --graph off
run b8_graph 400 python -u bench.py --batch-per-gpu 8 --steps 20 --warmup 5 --graph on
run b8_eager 400 python -u bench.py --batch-per-gpu 8 --steps 20 --warmup 5 --graph off
run fp32_b16 600 python -u bench.py --dtype fp32 --batch-per-gpu 16 --steps 5 --warmup 2
echo "[r3b] torchrun fp32"
timeout -k 10 600 python -u train-torchrun.py --model-ckpt t5-base --synthetic 256 --max-source-length 1024 \
  --max-target-length 128 --output-dir /tmp/ebench --batch-size 8 --grad-accum 2 --max-steps 6 --precision fp32 \
  --evaluation-steps 1000000 --max-eval-samples 4 > $O/torchrun_fp32.log 2>&1 || { tail -20 $O/torchrun_fp32.log; exit 1; }
grep -h "train_runtime\|\"loss\"" $O/torchrun_fp32.log | tail -3
