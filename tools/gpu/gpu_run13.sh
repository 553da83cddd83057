#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/ -q -m gpu -x > gpurun_out/gputests13.log 2>&1 || { echo GT_FAIL; grep -E "Error|assert|FAILED|passed|failed" gpurun_out/gputests13.log | tail -20; exit 1; }
tail -1 gpurun_out/gputests13.log
timeout -k 10 300 python bench.py > gpurun_out/bench13.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/bench13.log; exit 1; }
tail -1 gpurun_out/bench13.log | cut -c1-220
DLLM_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --batch-per-gpu 16 > gpurun_out/bench13_dp2.log 2>&1 || { echo DP2_FAIL; tail -30 gpurun_out/bench13_dp2.log; exit 1; }
grep '^{' gpurun_out/bench13_dp2.log | cut -c1-200
for occ in 2 3; do
DLLM_ATTN_OCC=$occ timeout -k 10 300 python tools/attn_bench.py > gpurun_out/attn13_occ$occ.jsonl 2>&1 || { echo AB_FAIL; tail -5 gpurun_out/attn13_occ$occ.jsonl; exit 1; }
echo "occ=$occ"; grep '^{' gpurun_out/attn13_occ$occ.jsonl | cut -c1-250
done
