#!/bin/bash
# Round 4: bias-gradient column sums on the side stream at large micro-batches (DLLM_BIAS_STREAM=1) vs inline (0),
# bart-large b=256, alternating; then the stream tests
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4z
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_grads_gpu.py -k "side_stream" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in 1 0; do
    DLLM_BIAS_STREAM=$v timeout -k 10 300 python bench.py --model bart-large --batch-per-gpu 256 --steps 8 --warmup 3 > $O/bart_b${v}_${r}.log 2>&1 || { tail -5 $O/bart_b${v}_${r}.log; exit 1; }
    echo "bias_stream=$v run $r: $(grep '"metric"' $O/bart_b${v}_${r}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
