#!/bin/bash
# Round 4: short-query dK/dV default (MB 4) vs off, bart-large b=256 and t5-base b=512, alternating, 3 reps
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4ae
mkdir -p $O
for r in 1 2 3; do
  for mb in 4 0; do
    DLLM_ATTN_DKDV_SQ_MB=$mb timeout -k 10 300 python bench.py --model bart-large --batch-per-gpu 256 --steps 8 --warmup 3 > $O/bart_mb${mb}_$r.log 2>&1 || { tail -5 $O/bart_mb${mb}_$r.log; exit 1; }
    echo "bart b256 MB=$mb $r: $(grep '"metric"' $O/bart_mb${mb}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
    DLLM_ATTN_DKDV_SQ_MB=$mb timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/t5_mb${mb}_$r.log 2>&1 || { tail -5 $O/t5_mb${mb}_$r.log; exit 1; }
    echo "t5 b512 MB=$mb $r: $(grep '"metric"' $O/t5_mb${mb}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
