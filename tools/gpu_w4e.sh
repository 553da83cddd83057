#!/bin/bash
# w4 staged-epilogue check: kernel tests, microbench (staged vs direct stores), whole-step A/B in one box.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/w4e
mkdir -p $O
echo "[w4e] tests"
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gemm_w4_gpu.py > $O/test.log 2>&1
rc=$?; [ $rc -gt 1 ] && { tail -40 $O/test.log; exit 1; }
grep -E "FAILED|passed|failed|Error" $O/test.log | tail -12
[ $rc -ne 0 ] && exit 1
echo "[w4e] microbench"
timeout -k 10 500 python -u tools/gemm_w4_bench.py --rounds 2 > $O/bench.jsonl 2>&1 || { tail -5 $O/bench.jsonl; exit 1; }
grep '^{' $O/bench.jsonl | python -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); print(f\"{r['shape']:14s} {r['phase']:5s} lib {r['lib_tflops']:7.1f} w4 {r['w4_tflops']:7.1f} rs1 {r['w4rs1_tflops']:7.1f} direct {r['w4direct_tflops']:7.1f}\")"
for i in 1 2; do
  for v in auto 1 0; do
    echo "[w4e] bench W4=$v #$i"
    DLLM_W4_GEMM=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/bench_${v}_$i.log 2>&1 || { tail -5 $O/bench_${v}_$i.log; exit 1; }
    echo "W4=$v $(grep -h '"metric"' $O/bench_${v}_$i.log | tail -1 | cut -c100-190)" | tee -a $O/ab.txt
  done
done
