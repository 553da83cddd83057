#!/bin/bash
# Round 4: weight gradients on a side stream (ops/streams.py): numerics + interleaved A/B at three batch sizes
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_grads_gpu.py -k "side_stream" tests/test_graph_gpu.py -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error" $O/tests.log | tail -20; [ $rc -eq 0 ] || exit 1
for r in 1 2; do
  for s in 1 0; do
    DLLM_WGRAD_STREAM=$s timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 > $O/b512_s$s.log 2>&1 || { tail -20 $O/b512_s$s.log; exit 1; }
    echo "b512 stream=$s: $(grep metric $O/b512_s$s.log | cut -c100-200)"
  done
done
for s in 1 0; do
  DLLM_WGRAD_STREAM=$s timeout -k 10 600 python -u bench.py --batch-per-gpu 8 --grad-accum 16 --steps 4 --warmup 2 > $O/b8_s$s.log 2>&1 || { tail -20 $O/b8_s$s.log; exit 1; }
  echo "b8xGA16 stream=$s: $(grep metric $O/b8_s$s.log | cut -c100-200)"
  DLLM_WGRAD_STREAM=$s timeout -k 10 600 python -u bench.py --batch-per-gpu 1 --steps 40 --warmup 3 > $O/b1_s$s.log 2>&1 || { tail -20 $O/b1_s$s.log; exit 1; }
  echo "b1 stream=$s: $(grep metric $O/b1_s$s.log | cut -c100-200)"
done
