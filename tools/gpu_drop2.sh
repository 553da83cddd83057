#!/bin/bash
# Packed-pair attention dropout: tests vs the CPU mirror, kernel and whole-step A/B against the previous build.
set -o pipefail
O=gpurun_out/drop2
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "attention or dropout" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
AB_TAIL=2 bash tools/ab_so.sh drop2/attn ab_so/old.so ab_so/new.so 2 python -u tools/attn_bench.py --quick || exit 1
bash tools/ab_so.sh drop2/bench ab_so/old.so ab_so/new.so 2 python bench.py --steps 10 --warmup 3 || exit 1
