#!/bin/bash
# whole-step A/B of the w4 routing (auto vs hipBLASLt-only), t5-base b=256 and bart-large b=64, one box.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/w4h
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gemm_w4_gpu.py -x > $O/test.log 2>&1 || { tail -20 $O/test.log; exit 1; }
tail -1 $O/test.log
for i in 1 2; do
  for v in auto 0; do
    DLLM_W4_GEMM=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/t5_${v}_$i.log 2>&1 || { tail -5 $O/t5_${v}_$i.log; exit 1; }
    echo "t5 W4=$v $(grep -h '"metric"' $O/t5_${v}_$i.log | tail -1 | cut -c100-190)" | tee -a $O/ab.txt
    DLLM_W4_GEMM=$v timeout -k 10 300 python -u bench.py --model bart-large --batch-per-gpu 64 --steps 6 --warmup 2 > $O/bart_${v}_$i.log 2>&1 || { tail -5 $O/bart_${v}_$i.log; exit 1; }
    echo "bart W4=$v $(grep -h '"metric"' $O/bart_${v}_$i.log | tail -1 | cut -c100-190)" | tee -a $O/ab.txt
  done
done
