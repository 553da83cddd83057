#!/bin/bash
# Round 4: short-query dK/dV kernel vs dkdv2 across batch sizes (T5 cross-attention shape: H 12, 128 x 1024 keys,
# key padding, dropout 0.1): MB forced to 2 / 4 vs off, to place the launcher's fill threshold
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4ai
mkdir -p $O
for B in 8 16 32 64 128; do
  for mb in 0 2 4; do
    tag=b${B}_mb$mb
    DLLM_ATTN_DKDV_SQ_MB=$mb DLLM_ATTN_DKDV_SQ_FORCE=1 ATTN_SQ=128 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/$tag -o run -- python tools/attn_cases.py $B 12 1024 0 1 0.1 1.0 6 > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; exit 1; }
    f=$(find $O/$tag -name "*.db" | head -n 1)
    python - "$f" "$tag" <<'PY'
import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
v = [float(d) for n, d in c.execute("select name, duration from kernels") if "dkdv" in n]
v = v[1:] if len(v) > 2 else v
print(f"{sys.argv[2]:>12}: dK/dV {sum(v) / len(v) / 1e3:8.1f} us")
PY
    find $O/$tag -name "*.db" -delete
  done
done
