#!/bin/bash
# Cost of the dropout hash in the FFN GEMM epilogue: fused forward at p = 0.1 vs p = 0 (same kernel, hash skipped).
set -o pipefail
O=gpurun_out/ffnhash
mkdir -p $O
for p in 0.1 0.0; do
  timeout -k 10 300 python -u tools/gemm_fused_bench.py --variants 8,9 --p $p --iters 20 > $O/p$p.log 2>&1 || { tail -5 $O/p$p.log; exit 1; }
  echo "== p=$p"; grep -v amdgpu.ids $O/p$p.log | cut -c1-300
done
