#!/bin/bash
# Round 4: per-feature cost of the attention kernels at full size (T5-base b=128 shape, BART-large b=64 shape)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4k
mkdir -p $O
for c in "t5full:128 12 1024 1 1 0.1 1.0" "t5nodrop:128 12 1024 1 1 0.0 1.0" "t5nobias:128 12 1024 0 1 0.1 1.0" "t5plain:128 12 1024 0 1 0.0 1.0" "t5plain_s8:128 12 1024 0 1 0.0 0.125" "bart:96 16 1024 0 1 0.0 0.125"; do
  tag=${c%%:*}; args=${c#*:}
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/$tag -o run -- python tools/attn_cases.py $args 5 > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; exit 1; }
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
    v = v[1:] if len(v) > 2 else v  # first call: cold
    print(f"  {sum(v) / len(v) / 1e3:9.1f} us x{len(v):>3}  {n[:100]}")
PY
  find $O/$tag -name "*.db" -delete
done
