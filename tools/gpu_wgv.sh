#!/bin/bash
# In-situ A/B of the weight-gradient kernel variants (csrc/gemm.hip) at the b=256 bench, one box.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/wgv
mkdir -p $O
for i in 1 2; do
  for v in 9 5 3 8; do
    DLLM_WGRAD_VARIANT=$v timeout -k 10 300 python -u bench.py --steps 8 --warmup 3 > $O/b_${v}_$i.log 2>&1 || { tail -5 $O/b_${v}_$i.log; exit 1; }
    echo "V=$v $(grep -h '"metric"' $O/b_${v}_$i.log | tail -1 | cut -c100-190)" | tee -a $O/ab.txt
  done
done
