#!/bin/bash
# Round 4: GELU backward GEMM persistent (DLLM_PP_PERSIST_DGELU=1) vs one tile per workgroup, bart-large b=256
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4ap
mkdir -p $O
DLLM_PP_PERSIST_DGELU=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "gelu_bwd_colsum or gemm_fused_backward" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in 1 0; do
    DLLM_PP_PERSIST_DGELU=$v timeout -k 10 300 python bench.py --model bart-large --batch-per-gpu 256 --steps 8 --warmup 3 > $O/bart_d${v}_$r.log 2>&1 || { tail -5 $O/bart_d${v}_$r.log; exit 1; }
    echo "dgelu_persist=$v $r: $(grep '"metric"' $O/bart_d${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
