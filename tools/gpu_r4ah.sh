#!/bin/bash
# Round 4 end: bench lines for the larger BASELINE configs and the new model types on the current tree
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4ah
mkdir -p $O
run() {  # tag model batch steps warmup [extra]
  local f=$O/$1.log
  timeout -k 10 400 python bench.py --model $2 --batch-per-gpu $3 --steps $4 --warmup $5 ${@:6} > $f 2>&1 || { tail -5 $f; return 1; }
  echo "$1: $(grep '"metric"' $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "samples/s", d["ms_per_step"], "ms/step", "mfu", d.get("mfu"))')"
}
run t5large_b32 t5-large 32 10 3 && run flant5xl_b16 flan-t5-xl 16 8 3 && run mt5base_b128 mt5-base 128 8 3 && run umt5base_b128 umt5-base 128 8 3 && run t5base_b8ga16 t5-base 8 4 2 --grad-accum 16
