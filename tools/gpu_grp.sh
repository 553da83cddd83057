#!/bin/bash
# w4 tile-group sweep (L2 reuse of the A panels) on the encoder forward / dgrad shapes.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/grp
mkdir -p $O
for g in 1 2 4 8 16; do
  echo "[grp] $g"
  timeout -k 10 300 python -u tools/gemm_w4_bench.py --rounds 2 --grp $g --only "enc" > $O/g$g.jsonl 2>&1 || { tail -5 $O/g$g.jsonl; exit 1; }
  grep '^{' $O/g$g.jsonl | python -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); print(f\"grp=$g {r['shape']:14s} {r['phase']:5s} lib {r['lib_tflops']:7.1f} w4rs1 {r['w4rs1_tflops']:7.1f}\")"
done
