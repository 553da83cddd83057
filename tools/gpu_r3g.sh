#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3g
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_beam_gpu.py tests/test_model_gpu.py -k "beam or kv or generat" > $O/test.log 2>&1
rc=$?; grep -E "FAILED|passed|failed|Error" $O/test.log | tail -8; [ $rc -ne 0 ] && { grep -E "^E " $O/test.log | head; exit 1; }
timeout -k 10 300 python -u tools/eval_bench.py --batch 818 --modes fused > $O/eval818.jsonl 2>&1 || { tail -20 $O/eval818.jsonl; exit 1; }
grep '^{' $O/eval818.jsonl
timeout -k 10 300 python -u tools/eval_bench.py --batch 256 --modes fused > $O/eval256.jsonl 2>&1 || { tail -20 $O/eval256.jsonl; exit 1; }
grep '^{' $O/eval256.jsonl
d=$O/evprof
mkdir -p $d
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d -o run -- python tools/eval_bench.py --batch 256 --n 256 --modes fused > $O/evprof.log 2>&1 || { tail -5 $O/evprof.log; exit 1; }
db=$(find $d -name "*.db" | head -n 1); csv=$(find $d -name "*kernel_stats.csv" | head -n 1)
python tools/prof_summary.py "${db:-$csv}" 1 > $O/evprof_summary.txt && head -30 $O/evprof_summary.txt
[ -n "$db" ] && rm -f "$db"
exit 0
