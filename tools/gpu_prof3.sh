#!/bin/bash
# Kernel profile of the final round-3 tree at the bench default (t5-base, per-GPU batch 512), summarised on the box.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/prof3
mkdir -p $O
d=/tmp/prof_b512
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $d -o run -- python bench.py --steps 2 --warmup 1 --graph off > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
python tools/prof_summary.py $(find $d -name "*.db" | head -n 1) 3 > $O/summary.txt || exit 1
grep -h '"metric"' $O/bench.log | cut -c1-200
head -22 $O/summary.txt
