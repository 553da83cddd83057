#!/bin/bash
# Context-parallel compute efficiency on one GPU (rank-0 share of the ring blocks vs the monolithic kernel).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/cp_bench.py --n 4096,8192,16384,32768 --w 1,2,4,8 > gpurun_out/cp58.jsonl 2> gpurun_out/cp58.err || { echo CP_FAIL; tail -20 gpurun_out/cp58.err; exit 1; }
cat gpurun_out/cp58.jsonl
timeout -k 10 300 python -u tools/cp_bench.py --n 8192,32768 --w 1,4,8 --p 0.1 > gpurun_out/cp58_p.jsonl 2>> gpurun_out/cp58.err || { echo CP_FAIL; tail -20 gpurun_out/cp58.err; exit 1; }
cat gpurun_out/cp58_p.jsonl
