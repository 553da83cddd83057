#!/bin/bash
# tune hipBLASLt/rocBLAS solutions for the other BASELINE configs' GEMM shapes, then re-measure them
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/tune20
for m in "bart-large 32" "t5-large 32" "flan-t5-xl 16"; do
  set -- $m
  DLLM_TUNABLEOP=tune DLLM_TUNABLEOP_DIR=gpurun_out/tune20/$1 timeout -k 10 600 python bench.py --model $1 --batch-per-gpu $2 --steps 1 --warmup 1 > gpurun_out/tune20_$1.log 2>&1 || { echo TUNE_FAIL $1; tail -5 gpurun_out/tune20_$1.log; exit 1; }
done
python tools/merge_tunableop.py gpurun_out/tune20/*/*.csv && cp configs/tunableop/gfx950.csv gpurun_out/gfx950_merged20.csv
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x -k "attention" > gpurun_out/gputests20.log 2>&1 || { echo GT_FAIL; grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/gputests20.log | tail -20; exit 1; }
tail -1 gpurun_out/gputests20.log
for m in "bart-large 32" "t5-large 32" "flan-t5-xl 16" "t5-base 64"; do
  set -- $m
  timeout -k 10 600 python bench.py --model $1 --batch-per-gpu $2 --steps 8 --warmup 3 > gpurun_out/bench20_$1.log 2>&1 || { echo BENCH_FAIL $1; tail -5 gpurun_out/bench20_$1.log; exit 1; }
  echo "$1 $(tail -1 gpurun_out/bench20_$1.log | cut -c1-200)"
done
