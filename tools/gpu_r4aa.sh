#!/bin/bash
# Round 4: dK/dV prologue with the K / V fragment loads issued before the key-mask reads (default build) vs after them
# (altso/_C_kvlate.so, -DDKDV_KV_EARLY=0): T5 cross-attention shape kernel times, then t5-base b=512 steps, alternating
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4aa
mkdir -p $O
for arm in early late; do
  if [ $arm = late ]; then export DLLM_NATIVE_SO=altso/_C_kvlate.so; else unset DLLM_NATIVE_SO; fi
  for c in "cross:512 12 1024 0 1 0.1 1.0" "self:128 12 1024 1 1 0.1 1.0"; do
    tag=${arm}_${c%%:*}; args=${c#*:}
    sq=""; [ ${c%%:*} = cross ] && sq=128
    ATTN_SQ=${sq:-1024} timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/$tag -o run -- python tools/attn_cases.py $args 5 > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; exit 1; }
    f=$(find $O/$tag -name "*.db" | head -n 1)
    echo "== $tag ($args)"
    python - "$f" <<'PY'
import sqlite3, sys
from collections import defaultdict
c = sqlite3.connect(sys.argv[1])
agg = defaultdict(list)
for n, d in c.execute("select name, duration from kernels"):
    if "attn" in n:
        agg[n].append(float(d))
for n, v in sorted(agg.items()):
    v = v[1:] if len(v) > 2 else v
    print(f"  {sum(v) / len(v) / 1e3:9.1f} us x{len(v):>3}  {n[:100]}")
PY
    find $O/$tag -name "*.db" -delete
  done
done
unset DLLM_NATIVE_SO
for r in 1 2; do
  for arm in early late; do
    if [ $arm = late ]; then export DLLM_NATIVE_SO=altso/_C_kvlate.so; else unset DLLM_NATIVE_SO; fi
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/b512_${arm}_$r.log 2>&1 || { tail -5 $O/b512_${arm}_$r.log; exit 1; }
    echo "b512 $arm $r: $(grep '"metric"' $O/b512_${arm}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
