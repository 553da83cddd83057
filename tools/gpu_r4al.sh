#!/bin/bash
# Round 4: dK/dV (dkdv2) with LDS-staged whole-row stores (default) vs per-lane stores (altso/_C_nostage2.so):
# numerics, kernel times (T5 encoder self-attention b=128, BART-large encoder b=64, T5 decoder self b=512), b=512 steps
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4al
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_model_gpu.py -k "attention or native_bf16 or context_parallel or chunked" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for arm in stage nostage; do
  if [ $arm = nostage ]; then export DLLM_NATIVE_SO=altso/_C_nostage2.so; else unset DLLM_NATIVE_SO; fi
  for c in "t5enc:128 12 1024 1 1 0.1 1.0:1024" "bartenc:64 16 1024 0 1 0.0 0.125:1024" "t5dec:512 12 128 1 0 0.1 1.0:128"; do
    name=${c%%:*}; rest=${c#*:}; args=${rest%%:*}; sq=${rest##*:}
    tag=${arm}_$name
    ATTN_SQ=$sq timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/$tag -o run -- python tools/attn_cases.py $args 5 > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; exit 1; }
    f=$(find $O/$tag -name "*.db" | head -n 1)
    python - "$f" "$tag" <<'PY'
import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
v = [float(d) for n, d in c.execute("select name, duration from kernels") if "dkdv" in n]
v = v[1:] if len(v) > 2 else v
print(f"{sys.argv[2]:>16}: dK/dV {sum(v) / len(v) / 1e3:8.1f} us")
PY
    find $O/$tag -name "*.db" -delete
  done
done
unset DLLM_NATIVE_SO
for r in 1 2; do
  for arm in stage nostage; do
    if [ $arm = nostage ]; then export DLLM_NATIVE_SO=altso/_C_nostage2.so; else unset DLLM_NATIVE_SO; fi
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/b512_${arm}_$r.log 2>&1 || { tail -5 $O/b512_${arm}_$r.log; exit 1; }
    echo "b512 $arm $r: $(grep '"metric"' $O/b512_${arm}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
