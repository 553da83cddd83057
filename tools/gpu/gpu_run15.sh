#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x -k "attention or native" > gpurun_out/gputests15.log 2>&1 || { echo GT_FAIL; grep -E "Error|assert|FAILED|passed|failed" gpurun_out/gputests15.log | tail -20; exit 1; }
tail -1 gpurun_out/gputests15.log
timeout -k 10 300 python tools/attn_bench.py > gpurun_out/attn15.jsonl 2>&1 || { echo AB_FAIL; tail -5 gpurun_out/attn15.jsonl; exit 1; }
grep '^{' gpurun_out/attn15.jsonl | cut -c1-250
timeout -k 10 600 python -m pytest tests/ -q -m gpu -x > gpurun_out/gputests15b.log 2>&1 || { echo GT_FAIL; grep -E "Error|assert|FAILED|passed|failed" gpurun_out/gputests15b.log | tail -20; exit 1; }
tail -1 gpurun_out/gputests15b.log
timeout -k 10 300 python bench.py > gpurun_out/bench15.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/bench15.log; exit 1; }
tail -1 gpurun_out/bench15.log | cut -c1-220
