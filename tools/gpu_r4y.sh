#!/bin/bash
# Round 4: weight-gradient split-K time model (default) vs the rounds-only model (DLLM_WGRAD_SPLIT_MODEL=rounds),
# alternating, graphed bench steps at batch 8, 1 and 512
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4y
mkdir -p $O
run() {  # model batch steps warmup rep
  local f=$O/b$2_$1_$5.log
  DLLM_WGRAD_SPLIT_MODEL=$1 timeout -k 10 300 python bench.py --batch-per-gpu $2 --steps $3 --warmup $4 > $f 2>&1 || { tail -5 $f; return 1; }
  echo "b$2 model=$1 rep $5: $(grep '"metric"' $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
for rep in 1 2; do
  run time 8 30 5 $rep && run rounds 8 30 5 $rep || exit 1
done
for rep in 1 2; do
  run time 1 40 10 $rep && run rounds 1 40 10 $rep || exit 1
done
run time 512 8 2 1 && run rounds 512 8 2 1 || exit 1
