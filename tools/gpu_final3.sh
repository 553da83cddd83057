#!/bin/bash
# End-of-round-3 re-measurement on the final tree: every GPU test, the default bench line, the other model configs and
# the reference-sized micro-batch lines (one JSON line each under gpurun_out/final3/).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/final3
mkdir -p $O
./tools/gpu_alltests.sh || exit 1
run() {
  name=$1; shift
  timeout -k 10 600 python -u bench.py "$@" > $O/$name.log 2>&1 || { tail -5 $O/$name.log; exit 1; }
  tail -1 $O/$name.log > $O/$name.json
  echo "$name $(python -c 'import json,sys; r=json.load(open(sys.argv[1])); print(r["value"], r["ms_per_step"], r["config"]["model"], r["config"]["per_gpu_batch"], r["config"].get("grad_accum"), r.get("mfu"))' $O/$name.json)"
}
run default --gpus 1 --steps 20 --warmup 5
run t5b_b256 --batch-per-gpu 256 --steps 10 --warmup 3
run bartl_b256 --model bart-large --batch-per-gpu 256 --steps 5 --warmup 2
run bartl_b32 --model bart-large --batch-per-gpu 32 --steps 10 --warmup 3
run t5l_b32 --model t5-large --batch-per-gpu 32 --steps 8 --warmup 3
run flanxl_b16 --model flan-t5-xl --batch-per-gpu 16 --steps 5 --warmup 2
run t5b_b8_graph --batch-per-gpu 8 --steps 20 --warmup 5
run t5b_b8ga16_graph --batch-per-gpu 8 --grad-accum 16 --steps 5 --warmup 2
run t5b_b1ga16_graph --batch-per-gpu 1 --grad-accum 16 --steps 5 --warmup 2
