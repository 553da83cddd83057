#!/bin/bash
# Saturated T5 bias tiles in the attention kernels: equivalence tests, attention microbench with / without,
# full GPU test suite, headline bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "attention or native_extension" --timeout 120 --timeout-method thread > gpurun_out/t30.log 2>&1 || { echo T_FAIL; grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/t30.log | tail -30; exit 1; }
tail -1 gpurun_out/t30.log
timeout -k 10 400 python -u tools/attn_bench.py > gpurun_out/ab30.jsonl 2> gpurun_out/ab30.err || { echo AB_FAIL; tail -20 gpurun_out/ab30.err; exit 1; }
cat gpurun_out/ab30.jsonl
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -x --timeout 180 --timeout-method thread > gpurun_out/g30.log 2>&1 || { echo G_FAIL; grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/g30.log | tail -30; exit 1; }
tail -1 gpurun_out/g30.log
timeout -k 10 300 python bench.py > gpurun_out/b30.log 2>&1 || { echo B_FAIL; tail -20 gpurun_out/b30.log; exit 1; }
tail -1 gpurun_out/b30.log
