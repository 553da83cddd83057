#!/bin/bash
# dK/dV LUT reads batched: attention tests, per-feature kernel times and whole-step A/B
# against the previous build (ab_so/old.so).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/fwdahead
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_grads_gpu.py \
  -k "attention or bias" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
AB_TAIL=1 bash tools/ab_so.sh fwdahead/attn ab_so/old.so ab_so/new.so 2 python -u tools/attn_bench.py --quick || exit 1
bash tools/ab_so.sh fwdahead/bench ab_so/old.so ab_so/new.so 2 python bench.py --steps 8 --warmup 3 || exit 1
