#!/bin/bash
# Round-3: beam kernel tests + eval re-time, small-batch graph vs eager, fp32 training lines.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3d
mkdir -p $O
echo "[r3d] beam tests"
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_beam_gpu.py > $O/test.log 2>&1
rc=$?; [ $rc -gt 1 ] && { tail -40 $O/test.log; exit 1; }
grep -E "FAILED|passed|failed|Error" $O/test.log | tail -12
echo "[r3d] eval"
timeout -k 10 400 python -u tools/eval_bench.py --batch 256 --modes fused,device > $O/eval.jsonl 2>&1 || { tail -20 $O/eval.jsonl; exit 1; }
grep '^{' $O/eval.jsonl
timeout -k 10 300 python -u tools/eval_bench.py --batch 818 --modes fused > $O/eval818.jsonl 2>&1 || { tail -20 $O/eval818.jsonl; exit 1; }
grep '^{' $O/eval818.jsonl
echo "[r3d] eval profile"
d=$O/evprof
mkdir -p $d
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d -o run -- python tools/eval_bench.py --batch 256 --n 256 --modes fused > $O/evprof.log 2>&1 || { tail -5 $O/evprof.log; exit 1; }
db=$(find $d -name "*.db" | head -n 1); csv=$(find $d -name "*kernel_stats.csv" | head -n 1)
python tools/prof_summary.py "${db:-$csv}" 1 > $O/evprof_summary.txt && head -30 $O/evprof_summary.txt
[ -n "$db" ] && rm -f "$db"
bash tools/gpu_r3b.sh
