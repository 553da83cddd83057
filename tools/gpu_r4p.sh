#!/bin/bash
# Round 4: dK/dV bias-gradient variant (ab_so/<variant>.so): attention numerics with it, then timing A/B vs default
set -o pipefail
O=gpurun_out/r4p
mkdir -p $O
v=$1
so=$(ls distributed_llms_example_amd/_C*.so | head -n 1)
cp "$so" /tmp/_C_keep.so
cp ab_so/$v.so "$so"
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attention" --timeout 300 --timeout-method thread > $O/tests_$v.log 2>&1
rc=$?
cp /tmp/_C_keep.so "$so"
tail -2 $O/tests_$v.log
[ $rc = 0 ] || exit $rc
bash tools/gpu_r4h.sh def $v
