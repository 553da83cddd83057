#!/bin/bash
# Full validation at the new bench default (per-GPU batch 128): GPU tests, smoke, bench, rocprofv3 stats, bart-large.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -q -m gpu -x --timeout 180 --timeout-method thread > gpurun_out/g52.log 2>&1 || { echo G_FAIL; grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/g52.log | tail -30; exit 1; }
tail -1 gpurun_out/g52.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke52.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/smoke52.log; exit 1; }
tail -1 gpurun_out/smoke52.log
timeout -k 10 300 python bench.py > gpurun_out/b52.log 2>&1 || { echo B_FAIL; tail -20 gpurun_out/b52.log; exit 1; }
tail -1 gpurun_out/b52.log
timeout -k 10 300 python bench.py --model bart-large --batch-per-gpu 32 > gpurun_out/b52_bart.log 2>&1 || { echo BB_FAIL; tail -20 gpurun_out/b52_bart.log; exit 1; }
tail -1 gpurun_out/b52_bart.log
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof52 -o prof -- python $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof52.log 2>&1 || { echo PROF_FAIL; tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof52.log; exit 1; }
tail -1 $GRAFT_REPO_ROOT/gpurun_out/prof52.log
