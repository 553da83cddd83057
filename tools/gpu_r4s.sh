#!/bin/bash
# Round 4: kernel profile of the t5-base batch-1 step (the reference's train-accelerator micro-batch), eager
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4s
mkdir -p $O
d=$O/prof_b1
mkdir -p $d
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $d -o run -- python bench.py --batch-per-gpu 1 --steps 4 --warmup 2 --graph off > $O/prof_b1.log 2>&1 || { tail -20 $O/prof_b1.log; exit 1; }
db=$(find $d -name "*.db" | head -n 1)
python tools/prof_summary.py "$db" 6 > $O/summary_b1.txt && head -30 $O/summary_b1.txt
python tools/trace_shapes.py "$db" 6 30 > $O/shapes_b1.txt && head -25 $O/shapes_b1.txt
find $d -name "*.db" -delete
