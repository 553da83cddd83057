#!/bin/bash
# Round 4: per-kernel profile of the bart-large b=256 step (eager) on the current tree
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4v
mkdir -p $O
d=$O/prof_bart
mkdir -p $d
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $d -o run -- python bench.py --model bart-large --batch-per-gpu 256 --steps 2 --warmup 1 --graph off > $O/prof_bart.log 2>&1 || { tail -20 $O/prof_bart.log; exit 1; }
db=$(find $d -name "*.db" | head -n 1)
python tools/prof_summary.py "$db" 3 > $O/summary_bart.txt && head -40 $O/summary_bart.txt
python tools/trace_shapes.py "$db" 3 40 > $O/shapes_bart.txt
find $d -name "*.db" -delete
