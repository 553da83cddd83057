#!/bin/bash
# Merged b=128 TunableOp table: full GPU test suite, smoke, bench x2, kernel-trace profile.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/p56
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 180 --timeout-method thread > gpurun_out/t56.log 2>&1 || { echo T_FAIL; grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/t56.log | tail -30; exit 1; }
tail -1 gpurun_out/t56.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke56.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/smoke56.log; exit 1; }
for i in 1 2; do
  timeout -k 10 300 python bench.py > gpurun_out/b56_$i.log 2>&1 || { echo B_FAIL; tail -20 gpurun_out/b56_$i.log; exit 1; }
  tail -1 gpurun_out/b56_$i.log
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/p56 -o run -- python bench.py --steps 3 --warmup 2 > gpurun_out/p56/log.txt 2>&1 || { echo P_FAIL; tail -20 gpurun_out/p56/log.txt; exit 1; }
find gpurun_out/p56 -name "*stats*"
