#!/bin/bash
# Round 4: per-shape kernel traces of bart-large b=256 and t5-base b=8 (eager steps)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4g
mkdir -p $O
for cfg in "bart256:--model bart-large --batch-per-gpu 256 --steps 2 --warmup 1 --graph off" "t5b8:--batch-per-gpu 8 --steps 2 --warmup 1 --graph off"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  d=$O/prof_$tag
  mkdir -p $d
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $d -o run -- python bench.py $args > $O/prof_$tag.log 2>&1 || { tail -20 $O/prof_$tag.log; exit 1; }
  db=$(find $d -name "*.db" | head -n 1)
  csv=$(find $d -name "*kernel_stats.csv" | head -n 1)
  python tools/prof_summary.py "${db:-$csv}" 3 > $O/summary_$tag.txt && head -24 $O/summary_$tag.txt
  tcsv=$(find $d -name "*kernel_trace.csv" | head -n 1)
  python tools/trace_shapes.py "${db:-$tcsv}" 3 60 > $O/shapes_$tag.txt && head -30 $O/shapes_$tag.txt
  find $d -name "*.db" -size +50M -delete
done
