#!/bin/bash
# After: fused FFN (v3), wgrad v9, saturated-bias backward tiles (forward path reverted): attention tests, attention
# microbench, headline bench, rocprofv3 kernel stats of the bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "attention or native_extension" --timeout 120 --timeout-method thread > gpurun_out/t31.log 2>&1 || { echo T_FAIL; grep -E "Error|error|assert|FAILED|passed|failed" gpurun_out/t31.log | tail -30; exit 1; }
tail -1 gpurun_out/t31.log
timeout -k 10 400 python -u tools/attn_bench.py --quick > gpurun_out/ab31.jsonl 2> gpurun_out/ab31.err || { echo AB_FAIL; tail -20 gpurun_out/ab31.err; exit 1; }
cat gpurun_out/ab31.jsonl
timeout -k 10 300 python bench.py > gpurun_out/b31.log 2>&1 || { echo B_FAIL; tail -20 gpurun_out/b31.log; exit 1; }
tail -1 gpurun_out/b31.log
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof31 -o prof -- python $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof31.log 2>&1 || { echo PROF_FAIL; tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof31.log; exit 1; }
tail -1 $GRAFT_REPO_ROOT/gpurun_out/prof31.log
