#!/bin/bash
# Eval re-time (shared cross K/V + one-gather cache reorder + fused beam step) and a b=256 step profile of the tree.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3f
mkdir -p $O
echo "[r3f] eval"
timeout -k 10 300 python -u tools/eval_bench.py --batch 818 --modes fused > $O/eval818.jsonl 2>&1 || { tail -20 $O/eval818.jsonl; exit 1; }
grep '^{' $O/eval818.jsonl
timeout -k 10 300 python -u tools/eval_bench.py --batch 256 --modes fused > $O/eval256.jsonl 2>&1 || { tail -20 $O/eval256.jsonl; exit 1; }
grep '^{' $O/eval256.jsonl
d=$O/evprof
mkdir -p $d
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d -o run -- python tools/eval_bench.py --batch 256 --n 256 --modes fused > $O/evprof.log 2>&1 || { tail -5 $O/evprof.log; exit 1; }
db=$(find $d -name "*.db" | head -n 1); csv=$(find $d -name "*kernel_stats.csv" | head -n 1)
python tools/prof_summary.py "${db:-$csv}" 1 > $O/evprof_summary.txt && head -24 $O/evprof_summary.txt
[ -n "$db" ] && rm -f "$db"
echo "[r3f] bench + profile b256 (eager profile, 4 steps)"
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
grep -h '"metric"' $O/bench.log | cut -c1-200
d=$O/prof
mkdir -p $d
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d -o run -- python bench.py --steps 3 --warmup 1 --graph off > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
db=$(find $d -name "*.db" | head -n 1); csv=$(find $d -name "*kernel_stats.csv" | head -n 1)
python tools/prof_summary.py "${db:-$csv}" 4 > $O/prof_summary.txt && head -40 $O/prof_summary.txt
[ -n "$db" ] && rm -f "$db"
exit 0
