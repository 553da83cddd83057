#!/bin/bash
# w4 GEMM re-check after the persistent-store fix: tests, microbench, whole-step A/B (hipBLASLt vs w4 RS=0/1).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/w4d
mkdir -p $O
step() { echo "[w4d] $*"; }
step tests
timeout -k 10 700 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gemm_w4_gpu.py \
  tests/test_model_gpu.py tests/test_graph_gpu.py tests/test_kernels_gpu.py tests/test_grads_gpu.py -s > $O/test.log 2>&1
rc=$?; [ $rc -gt 1 ] && { tail -40 $O/test.log; exit 1; }
grep -E "FAILED|passed|failed|Error" $O/test.log | tail -15
grep -E "^\[parity" $O/test.log | head
step microbench
timeout -k 10 400 python -u tools/gemm_w4_bench.py --rounds 2 > $O/bench.jsonl 2>&1 || { tail -5 $O/bench.jsonl; exit 1; }
cut -c1-330 $O/bench.jsonl
for v in "0 0" "1 0" "1 1" "0 0" "1 0" "1 1"; do
  set -- $v
  step bench W4=$1 RS=$2
  DLLM_W4_GEMM=$1 DLLM_W4_RS=$2 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/bench_$1_$2.log 2>&1 || { tail -5 $O/bench_$1_$2.log; exit 1; }
  echo "W4=$1 RS=$2 $(tail -1 $O/bench_$1_$2.log | cut -c1-160)" | tee -a $O/ab.txt
done
