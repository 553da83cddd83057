#!/bin/bash
# GPU tests (fused wgrad / stacked cross-KV paths) + re-tune new GEMM shapes + bench + kernel profile
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/tune10
timeout -k 10 600 python -m pytest tests/ -q -m gpu -x > gpurun_out/gputests10.log 2>&1 || { echo GT_FAIL; grep -E "Error|assert|FAILED|passed|failed" gpurun_out/gputests10.log | tail -20; exit 1; }
tail -1 gpurun_out/gputests10.log
for b in 64 32; do
DLLM_TUNABLEOP=tune DLLM_TUNABLEOP_DIR=gpurun_out/tune10/b$b timeout -k 10 600 python bench.py --steps 1 --warmup 1 --batch-per-gpu $b > gpurun_out/tune10_b$b.log 2>&1 || { echo TUNE_FAIL; tail -20 gpurun_out/tune10_b$b.log; exit 1; }
done
python tools/merge_tunableop.py gpurun_out/tune10/b64/*.csv gpurun_out/tune10/b32/*.csv && cp configs/tunableop/gfx950.csv gpurun_out/gfx950_merged10.csv
for b in 64 32; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --batch-per-gpu $b > gpurun_out/bench10_b$b.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/bench10_b$b.log; exit 1; }
  tail -1 gpurun_out/bench10_b$b.log | cut -c1-200
done
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof10 -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --batch-per-gpu 64 > $R/gpurun_out/prof10.log 2>&1 || { echo PROF_FAIL; tail -20 $R/gpurun_out/prof10.log; exit 1; }
rm -f $R/gpurun_out/prof10/run_kernel_trace.csv
python3 $R/tools/prof_summary.py $R/gpurun_out/prof10/run_kernel_stats.csv 7 > $R/gpurun_out/prof10_summary.txt; head -45 $R/gpurun_out/prof10_summary.txt
