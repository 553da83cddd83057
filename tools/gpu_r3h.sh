#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3h
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_beam_gpu.py > $O/test.log 2>&1
rc=$?; grep -E "FAILED|passed|failed|Error" $O/test.log | tail -8; [ $rc -ne 0 ] && { grep -E "^E " $O/test.log | head; exit 1; }
timeout -k 10 300 python -u tools/eval_bench.py --batch 818 --modes fused,device > $O/eval818.jsonl 2>&1 || { tail -20 $O/eval818.jsonl; exit 1; }
grep '^{' $O/eval818.jsonl
timeout -k 10 300 python -u tools/eval_bench.py --batch 256 --modes fused > $O/eval256.jsonl 2>&1 || { tail -20 $O/eval256.jsonl; exit 1; }
grep '^{' $O/eval256.jsonl
echo "[r3h] gloo 2 ranks on one GPU"
bash tools/gloo2_gpu.sh
