#!/bin/bash
# Round 4: staged GELU / gated-GELU backward epilogues (default) vs per-lane (altso/_C_bwdnostage.so,
# -DPP_STAGE_BWD=0): numerics, then flan-t5-base b=128 and bart-large b=256 steps, alternating
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4as
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_grads_gpu.py -k "gemm_fused or geglu or gelu_bwd or native_bf16 or fused_ffn or fp32_training" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for arm in stage nostage; do
    if [ $arm = nostage ]; then export DLLM_NATIVE_SO=altso/_C_bwdnostage.so; else unset DLLM_NATIVE_SO; fi
    timeout -k 10 300 python bench.py --model flan-t5-base --batch-per-gpu 128 --steps 8 --warmup 3 > $O/flan_${arm}_$r.log 2>&1 || { tail -5 $O/flan_${arm}_$r.log; exit 1; }
    echo "flan-t5-base b128 $arm $r: $(grep '"metric"' $O/flan_${arm}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
    timeout -k 10 300 python bench.py --model bart-large --batch-per-gpu 256 --steps 8 --warmup 3 > $O/bart_${arm}_$r.log 2>&1 || { tail -5 $O/bart_${arm}_$r.log; exit 1; }
    echo "bart b256 $arm $r: $(grep '"metric"' $O/bart_${arm}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
