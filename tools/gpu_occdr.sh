#!/bin/bash
# Cross-attention dK/dV at 3 workgroups per CU (NB=2 ring, 168 VGPRs) vs 2 (NB=3): kernel and whole-step A/B.
set -o pipefail
O=gpurun_out/occdr
mkdir -p $O
DLLM_ATTN_DKDV_OCC_DR=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py -k "attention" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for v in 0 1; do
    DLLM_ATTN_DKDV_OCC_DR=$v timeout -k 10 300 python -u tools/attn_anat.py --S 1024 --cfg b0k1d1 --iters 5 > /dev/null 2>&1 || true
    DLLM_ATTN_DKDV_OCC_DR=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/b${v}_$i.log 2>&1 || { tail -5 $O/b${v}_$i.log; exit 1; }
    echo "occdr=$v $(tail -1 $O/b${v}_$i.log | cut -c1-190)"
  done
done
mkdir -p $O/prof0 $O/prof1
for v in 0 1; do
  DLLM_ATTN_DKDV_OCC_DR=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof$v -o run -- python bench.py --steps 2 --warmup 1 --graph off > $O/prof$v/log 2>&1 || { tail -5 $O/prof$v/log; exit 1; }
done
