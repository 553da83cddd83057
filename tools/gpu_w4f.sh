#!/bin/bash
# w4 FFN epilogues: kernel tests, model tests, whole-step A/B (DLLM_W4_FFN 0 / 1) in one box.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/w4f
mkdir -p $O
echo "[w4f] tests"
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gemm_w4_gpu.py tests/test_model_gpu.py tests/test_graph_gpu.py > $O/test.log 2>&1
rc=$?; [ $rc -gt 1 ] && { tail -40 $O/test.log; exit 1; }
grep -E "FAILED|passed|failed|Error" $O/test.log | tail -12
[ $rc -ne 0 ] && { grep -E "^E " $O/test.log | head -20; exit 1; }
for i in 1 2; do
  for v in 1 0; do
    echo "[w4f] bench W4_FFN=$v #$i"
    DLLM_W4_FFN=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/bench_${v}_$i.log 2>&1 || { tail -5 $O/bench_${v}_$i.log; exit 1; }
    echo "W4_FFN=$v $(grep -h '"metric"' $O/bench_${v}_$i.log | tail -1 | cut -c100-190)" | tee -a $O/ab.txt
  done
done
