#!/bin/bash
# Re-validate after container re-creation: GPU tests, smoke, bench, rocprof kernel stats.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/gputests27.log 2>&1 || { echo GT_FAIL; grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/gputests27.log | tail -20; exit 1; }
tail -1 gpurun_out/gputests27.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke27.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/smoke27.log; exit 1; }
tail -1 gpurun_out/smoke27.log
timeout -k 10 300 python bench.py > gpurun_out/bench27.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/bench27.log; exit 1; }
tail -1 gpurun_out/bench27.log
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof27 -o prof -- python $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof27.log 2>&1 || { echo PROF_FAIL; tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof27.log; exit 1; }
tail -1 $GRAFT_REPO_ROOT/gpurun_out/prof27.log
