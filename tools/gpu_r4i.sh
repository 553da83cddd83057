#!/bin/bash
# Round 4: pipelined dK/dV kernel — attention numerics tests, then timing A/B against the staged build (ab_so/)
set -o pipefail
O=gpurun_out/r4i
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_grads_gpu.py -x -q -k "attention or attn" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/gpu_r4h.sh "$@"
