#!/bin/bash
# Round 4: kernel profile of the t5-base batch-8 micro-step (the reference's torchrun micro-batch scale), eager, GA 1
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4x
mkdir -p $O
d=$O/prof_b8
mkdir -p $d
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $d -o run -- python bench.py --batch-per-gpu 8 --steps 6 --warmup 2 --graph off > $O/prof_b8.log 2>&1 || { tail -20 $O/prof_b8.log; exit 1; }
db=$(find $d -name "*.db" | head -n 1)
python tools/prof_summary.py "$db" 8 > $O/summary_b8.txt && head -40 $O/summary_b8.txt
python tools/trace_shapes.py "$db" 8 40 > $O/shapes_b8.txt
find $d -name "*.db" -delete
timeout -k 10 300 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5 > $O/bench_b8.log 2>&1 || { tail -5 $O/bench_b8.log; exit 1; }
grep metric $O/bench_b8.log | cut -c1-400
