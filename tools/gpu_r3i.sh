#!/bin/bash
# Round-3 validation on the current tree: every GPU test, the two-rank gloo rehearsal of the multi-rank bench /
# Trainer paths, smoke(), and a kernel profile of the default bench step.
set -o pipefail
export TMPDIR=/tmp
./tools/gpu_alltests.sh || exit 1
./tools/gloo2_gpu.sh || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -2 || exit 1
mkdir -p gpurun_out/prof_r3i
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r3i -o run -- python bench.py --steps 3 --warmup 1 --graph off > gpurun_out/prof_r3i/bench.log 2>&1 || { tail -5 gpurun_out/prof_r3i/bench.log; exit 1; }
tail -1 gpurun_out/prof_r3i/bench.log | cut -c1-200
