#!/bin/bash
# Round 4: short-query dK/dV kernel with the adaptive key-block count — numerics (attention + model tests), then
# t5-base b=512 and bart-large b=256 steps, default vs DLLM_ATTN_DKDV_SQ_MB=0, alternating
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4ac
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_model_gpu.py -k "attention or native_bf16 or fp32_training" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for mb in 8 0; do
    DLLM_ATTN_DKDV_SQ_MB=$mb timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/t5_mb${mb}_$r.log 2>&1 || { tail -5 $O/t5_mb${mb}_$r.log; exit 1; }
    echo "t5 b512 MB=$mb $r: $(grep '"metric"' $O/t5_mb${mb}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
for r in 1 2; do
  for mb in 8 0; do
    DLLM_ATTN_DKDV_SQ_MB=$mb timeout -k 10 300 python bench.py --model bart-large --batch-per-gpu 256 --steps 8 --warmup 3 > $O/bart_mb${mb}_$r.log 2>&1 || { tail -5 $O/bart_mb${mb}_$r.log; exit 1; }
    echo "bart b256 MB=$mb $r: $(grep '"metric"' $O/bart_mb${mb}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
