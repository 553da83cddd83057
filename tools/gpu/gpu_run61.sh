#!/bin/bash
# Kernel profile of a 32K-token t5-base training step (chunked encoder attention, key-chunked cross-attention).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/p61
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/p61 -o run -- python bench.py --batch-per-gpu 1 --src-len 32768 --steps 2 --warmup 1 > gpurun_out/p61/log.txt 2>&1 || { echo P_FAIL; tail -20 gpurun_out/p61/log.txt; exit 1; }
tail -1 gpurun_out/p61/log.txt
python tools/prof_summary.py gpurun_out/p61/run_results.db 3 > gpurun_out/p61/summary.txt
rm -f gpurun_out/p61/run_results.db
