#!/bin/bash
# Round 4: ping-pong GEMM store-only epilogues staged through LDS as whole-row stores (default) vs per-lane stores
# (altso/_C_ppnostage.so, -DPP_STAGE=0): fused-GEMM numerics, in-step kernel times, t5-base b=512 / bart-large b=256
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4an
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_grads_gpu.py -k "gemm_fused or gemm_pp or relu_bit or geglu or native_bf16 or fused_ffn or ffn" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for arm in stage nostage; do
  if [ $arm = nostage ]; then export DLLM_NATIVE_SO=altso/_C_ppnostage.so; else unset DLLM_NATIVE_SO; fi
  d=$O/p_$arm
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d -o run -- python bench.py --steps 2 --warmup 1 --graph off > $O/p_$arm.log 2>&1 || { tail -5 $O/p_$arm.log; exit 1; }
  f=$(find $d -name "*.db" | head -n 1)
  python - "$f" "$arm" <<'PY'
import sqlite3, sys
from collections import defaultdict
c = sqlite3.connect(sys.argv[1])
agg = defaultdict(float); tot = 0.0
for n, d in c.execute("select name, duration from kernels"):
    tot += float(d)
    if "gemm_pp" in n: agg[n[:70]] += float(d)
print(f"== {sys.argv[2]}: total {tot / 3e6:.2f} ms/step")
for k, v in sorted(agg.items()): print(f"   {v / 3e6:7.2f} ms/step  {k}")
PY
  find $d -name "*.db" -delete
done
unset DLLM_NATIVE_SO
for r in 1 2; do
  for arm in stage nostage; do
    if [ $arm = nostage ]; then export DLLM_NATIVE_SO=altso/_C_ppnostage.so; else unset DLLM_NATIVE_SO; fi
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/t5_${arm}_$r.log 2>&1 || { tail -5 $O/t5_${arm}_$r.log; exit 1; }
    echo "t5 b512 $arm $r: $(grep '"metric"' $O/t5_${arm}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
    timeout -k 10 300 python bench.py --model bart-large --batch-per-gpu 256 --steps 8 --warmup 3 > $O/bart_${arm}_$r.log 2>&1 || { tail -5 $O/bart_${arm}_$r.log; exit 1; }
    echo "bart b256 $arm $r: $(grep '"metric"' $O/bart_${arm}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
