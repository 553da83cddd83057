#!/bin/bash
# Round 4: short-query dK/dV kernel (attn_bwd_dkdv_sq_kernel, DLLM_ATTN_DKDV_SQ_MB) — numerics, kernel times on the T5
# cross-attention shape for MB = 0 (dkdv2) / 2 / 4 / 8, then t5-base b=512 steps MB 4 vs 0, alternating
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4ab
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "attention" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for mb in 0 2 4 8; do
  tag=mb$mb
  DLLM_ATTN_DKDV_SQ_MB=$mb ATTN_SQ=128 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/$tag -o run -- python tools/attn_cases.py 512 12 1024 0 1 0.1 1.0 5 > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; exit 1; }
  f=$(find $O/$tag -name "*.db" | head -n 1)
  echo "== MB $mb"
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
for r in 1 2; do
  for mb in 4 0; do
    DLLM_ATTN_DKDV_SQ_MB=$mb timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/b512_mb${mb}_$r.log 2>&1 || { tail -5 $O/b512_mb${mb}_$r.log; exit 1; }
    echo "b512 MB=$mb $r: $(grep '"metric"' $O/b512_mb${mb}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
