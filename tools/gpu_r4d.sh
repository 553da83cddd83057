#!/bin/bash
# Round 4: full GPU test suite + the bench lines (default, fp32, bart-large, accelerator b1) on one box
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4d
mkdir -p $O
timeout -k 10 1500 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -25
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
echo "default: $(grep metric $O/bench.log | cut -c100-300)"
timeout -k 10 600 python -u bench.py --dtype fp32 --batch-per-gpu 16 --steps 6 --warmup 2 > $O/fp32.log 2>&1 || { tail -20 $O/fp32.log; exit 1; }
echo "fp32: $(grep metric $O/fp32.log | cut -c100-300)"
timeout -k 10 600 python -u bench.py --model bart-large --steps 8 --warmup 3 > $O/bart.log 2>&1 || { tail -20 $O/bart.log; exit 1; }
echo "bart: $(grep metric $O/bart.log | cut -c1-300)"
