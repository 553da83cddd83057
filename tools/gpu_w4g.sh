#!/bin/bash
# w4 ReLU backward on the ping-pong forward's mask: tests + whole-step A/B (DLLM_W4_FFN_BWD 1 / 0) on one box.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/w4g
mkdir -p $O
echo "[w4g] tests"
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gemm_w4_gpu.py tests/test_model_gpu.py tests/test_grads_gpu.py > $O/test.log 2>&1
rc=$?; [ $rc -gt 1 ] && { tail -40 $O/test.log; exit 1; }
grep -E "FAILED|passed|failed|Error" $O/test.log | tail -12
[ $rc -ne 0 ] && { grep -E "^E " $O/test.log | head -20; exit 1; }
for i in 1 2 3; do
  for v in 1 0; do
    DLLM_W4_FFN_BWD=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/bench_${v}_$i.log 2>&1 || { tail -5 $O/bench_${v}_$i.log; exit 1; }
    echo "W4_FFN_BWD=$v $(grep -h '"metric"' $O/bench_${v}_$i.log | tail -1 | cut -c100-190)" | tee -a $O/ab.txt
  done
done
