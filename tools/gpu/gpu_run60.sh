#!/bin/bash
# Full GPU suite + smoke + headline bench after the context-parallel / long-sequence work.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/t60.log 2>&1 || { echo T_FAIL; grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/t60.log | tail -30; exit 1; }
tail -1 gpurun_out/t60.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke60.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/smoke60.log; exit 1; }
echo smoke ok
timeout -k 10 300 python bench.py > gpurun_out/b60.log 2>&1 || { echo B_FAIL; tail -20 gpurun_out/b60.log; exit 1; }
tail -1 gpurun_out/b60.log
