#!/bin/bash
# Round 4 end-of-session: per-shape kernel trace of the t5-base b=512 step (eager) + three bench lines of the final tree
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4ag
mkdir -p $O
d=$O/prof_b512
mkdir -p $d
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $d -o run -- python bench.py --steps 2 --warmup 1 --graph off > $O/prof_b512.log 2>&1 || { tail -20 $O/prof_b512.log; exit 1; }
db=$(find $d -name "*.db" | head -n 1)
python tools/prof_summary.py "$db" 3 > $O/summary_b512.txt && head -24 $O/summary_b512.txt
python tools/trace_shapes.py "$db" 3 40 > $O/shapes_b512.txt
find $d -name "*.db" -delete
for i in 1 2 3; do
  timeout -k 10 600 python -u bench.py --steps 12 --warmup 3 > $O/bench_$i.log 2>&1 || { tail -20 $O/bench_$i.log; exit 1; }
  echo "bench $i: $(grep metric $O/bench_$i.log | cut -c100-200)"
done
