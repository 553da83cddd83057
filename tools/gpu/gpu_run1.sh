#!/bin/bash
# smoke + bench sweep + rocprof kernel stats
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
for b in 16 32 64; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --batch-per-gpu $b > gpurun_out/bench_b$b.log 2>&1 || { echo BENCH_FAIL $b; tail -30 gpurun_out/bench_b$b.log; exit 1; }
  tail -1 gpurun_out/bench_b$b.log
done
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof1 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --batch-per-gpu 32 > $GRAFT_REPO_ROOT/gpurun_out/prof1.log 2>&1 || { echo PROF_FAIL; tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof1.log; exit 1; }
echo PROF_OK
