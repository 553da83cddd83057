#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -k "gemm_wgrad or colsum" > gpurun_out/gemm21_tests.log 2>&1 || { echo GT_FAIL; grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/gemm21_tests.log | tail -20; exit 1; }
tail -1 gpurun_out/gemm21_tests.log
timeout -k 10 300 python tools/gemm_bench.py --variants 0,3,1,4,5,6 --no-torch --shapes 65536:768:768,65536:2304:768,65536:3072:768,65536:768:3072,65536:18432:768,8192:3072:768 > gpurun_out/gemm21_bench.jsonl 2>&1 || { echo GB_FAIL; tail -20 gpurun_out/gemm21_bench.jsonl; exit 1; }
grep '^{' gpurun_out/gemm21_bench.jsonl
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU -d $R/gpurun_out/pmc21a -o run --output-format csv -- python3 $R/tools/gemm_bench.py --shapes 65536:3072:768 --variants 0 --iters 3 --no-torch > $R/gpurun_out/pmc21a.log 2>&1 || { echo PMC_FAIL; tail -20 $R/gpurun_out/pmc21a.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES -d $R/gpurun_out/pmc21b -o run --output-format csv -- python3 $R/tools/gemm_bench.py --shapes 65536:3072:768 --variants 0 --iters 3 --no-torch > $R/gpurun_out/pmc21b.log 2>&1 || { echo PMC_FAIL; tail -20 $R/gpurun_out/pmc21b.log; exit 1; }
ls $R/gpurun_out/pmc21a $R/gpurun_out/pmc21b
cd $R
for m in "bart-large 32" "t5-large 32" "t5-base 64"; do
  set -- $m
  timeout -k 10 600 python bench.py --model $1 --batch-per-gpu $2 --steps 8 --warmup 3 > gpurun_out/bench21_$1.log 2>&1 || { echo BENCH_FAIL $1; tail -5 gpurun_out/bench21_$1.log; exit 1; }
  echo "$1 $(tail -1 gpurun_out/bench21_$1.log | cut -c1-200)"
done
