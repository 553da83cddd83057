#!/bin/bash
# Per-kernel profile of the t5-base b=256 step with the T5 FFN on w4 epilogues vs the ping-pong kernels (eager, 3 steps).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ffnprof
mkdir -p $O
for v in 1 0; do
  d=$O/p$v
  mkdir -p $d
  echo "[ffnprof] W4_FFN=$v"
  DLLM_W4_FFN=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d -o run -- python bench.py --steps 3 --warmup 1 --graph off > $O/p$v.log 2>&1 || { tail -5 $O/p$v.log; exit 1; }
  db=$(find $d -name "*.db" | head -n 1); csv=$(find $d -name "*kernel_stats.csv" | head -n 1)
  python tools/prof_summary.py "${db:-$csv}" 4 > $O/p${v}_summary.txt && grep -E "gemm_pp|gemm_w4|Cijk|total" $O/p${v}_summary.txt | head -14
  [ -n "$db" ] && rm -f "$db"
done
exit 0
