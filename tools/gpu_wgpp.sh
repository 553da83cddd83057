#!/bin/bash
# wgrad variant 10 (staggered wave groups): bitwise / numerics tests, then whole-step A/B against the default (9).
set -o pipefail
O=gpurun_out/wgpp
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "gemm_wgrad" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for v in 9 11; do
    DLLM_WGRAD_VARIANT=$v timeout -k 10 300 python bench.py --steps 8 --warmup 3 > $O/b${v}_$i.log 2>&1 || { tail -5 $O/b${v}_$i.log; exit 1; }
    echo "V=$v $(tail -1 $O/b${v}_$i.log | cut -c1-190)"
  done
done
