#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/tune
export TMPDIR=/tmp
timeout -k 10 300 python tools/hf_comparator.py --prec bf16-amp --batch 64 >> gpurun_out/hf_comparator_b64.jsonl 2>gpurun_out/hf64.err || echo HF64_FAIL
tail -1 gpurun_out/hf_comparator_b64.jsonl
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tune/tunableop_results%d.csv PYTORCH_TUNABLEOP_VERBOSE=0
timeout -k 10 900 python bench.py --steps 5 --warmup 2 --batch-per-gpu 32 > gpurun_out/bench_tune_b32.log 2>&1 || { echo TUNE_FAIL; tail -20 gpurun_out/bench_tune_b32.log; exit 1; }
tail -1 gpurun_out/bench_tune_b32.log
export PYTORCH_TUNABLEOP_TUNING=0
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --batch-per-gpu 32 > gpurun_out/bench_tuned_b32.log 2>&1 || { echo TUNED_FAIL; tail -20 gpurun_out/bench_tuned_b32.log; exit 1; }
tail -1 gpurun_out/bench_tuned_b32.log
ls -la gpurun_out/tune
