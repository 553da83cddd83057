#!/bin/bash
# HF comparator at per-GPU batch 128 (bf16 autocast, SDPA) — the reference stack at the new bench batch.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/hf_comparator.py --batch 128 --steps 5 --warmup 2 --prec bf16-amp --attn sdpa > gpurun_out/hf51.log 2>&1 || { echo HF_FAIL; grep -iE "memory|error" gpurun_out/hf51.log | tail -3; }
tail -2 gpurun_out/hf51.log
