#!/bin/bash
# Round 4: in-step kernel time of the T5 cross-attention dK/dV (eager b=512 step under rocprofv3), MB = 4 / 8 / 0
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4aq
mkdir -p $O
for mb in 4 8; do
  d=$O/p$mb
  DLLM_ATTN_DKDV_SQ_MB=$mb timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d -o run -- python bench.py --steps 2 --warmup 1 --graph off > $O/p$mb.log 2>&1 || { tail -5 $O/p$mb.log; exit 1; }
  f=$(find $d -name "*.db" | head -n 1)
  echo "== MB $mb"
  python - "$f" <<'PY'
import sqlite3, sys
from collections import defaultdict
c = sqlite3.connect(sys.argv[1])
agg = defaultdict(list)
tot = 0.0
for n, d in c.execute("select name, duration from kernels"):
    tot += float(d)
    if "attn_bwd_dkdv" in n or "attn_bwd_dq" in n:
        agg[n[:90]].append(float(d))
print(f"  total kernel time {tot / 3e6:.2f} ms/step")
for n, v in sorted(agg.items()):
    print(f"  {sum(v) / 3e6:8.2f} ms/step  {len(v) / 3:5.1f} calls/step  {n}")
PY
  find $d -name "*.db" -delete
done
