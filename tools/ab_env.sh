#!/bin/bash
# A/B bench on one box: alternate two env settings (VAR=A / VAR=B), two rounds each.
#   bash tools/ab_env.sh TAG "ENV_A" "ENV_B" [bench args]
set -o pipefail
tag=$1; ea=$2; eb=$3; shift 3
mkdir -p gpurun_out/$tag
for i in 1 2; do
  for side in A B; do
    e=$ea; [ $side = B ] && e=$eb
    env $e timeout -k 10 300 python bench.py "$@" > gpurun_out/$tag/${side}_$i.log 2>&1 || { tail -5 gpurun_out/$tag/${side}_$i.log; exit 1; }
    echo "$side($e) $(tail -1 gpurun_out/$tag/${side}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("peak_mem_gb"))')"
  done
done
