#!/bin/bash
# Round 4: per-GPU batch 512 vs 640 (t5-base bench default), interleaved, with peak memory
set -o pipefail
O=gpurun_out/r4r
mkdir -p $O
for i in 1 2; do
  for b in 512 640; do
    timeout -k 10 600 python -u bench.py --batch-per-gpu $b --steps 10 --warmup 3 > $O/b${b}_$i.log 2>&1 || { tail -20 $O/b${b}_$i.log; exit 1; }
    echo "b$b: $(grep metric $O/b${b}_$i.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('peak_mem_gb', d.get('config',{}).get('peak_mem_gb')))")"
  done
done
