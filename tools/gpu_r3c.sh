#!/bin/bash
# Round-3 check: model-level GPU tests, whole-step A/B (GEMM routing, LM-head chunked vs full), b=256 kernel profile.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3c
mkdir -p $O
echo "[r3c] tests"
timeout -k 10 500 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_model_gpu.py \
  tests/test_grads_gpu.py -s > $O/test.log 2>&1
rc=$?; [ $rc -gt 1 ] && { tail -40 $O/test.log; exit 1; }
grep -E "FAILED|passed|failed|parity|fused-ffn" $O/test.log | tail -25
run() {  # tag, env..., -- implied: bench args fixed
  local tag=$1; shift
  echo "[r3c] $tag"
  env "$@" timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/$tag.log 2>&1 || { echo "[r3c] $tag failed rc=$?"; tail -15 $O/$tag.log; exit 1; }
  echo "$tag $(grep -h '"metric"' $O/$tag.log | tail -1 | cut -c100-190)" | tee -a $O/ab.txt
}
for i in 1 2; do
  run w4auto_$i DLLM_W4_GEMM=auto
  run w4off_$i DLLM_W4_GEMM=0
  run lmfull_$i DLLM_LMHEAD_FULL_MB=-1
done
echo "[r3c] profile b256"
d=$O/prof
mkdir -p $d
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $d -o run -- python bench.py --steps 3 --warmup 2 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
db=$(find $d -name "*.db" | head -n 1); csv=$(find $d -name "*kernel_stats.csv" | head -n 1)
python tools/prof_summary.py "${db:-$csv}" 5 > $O/prof_summary.txt && head -45 $O/prof_summary.txt
[ -n "$db" ] && rm -f "$db"
exit 0
