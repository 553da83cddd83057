#!/bin/bash
# Round-3: w4 main-loop ablations, LM-head chunked vs full, BART norm-colsum A/B, per-model bench lines.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3e
mkdir -p $O
echo "[r3e] w4 ablations"
timeout -k 10 300 python -u tools/gemm_w4_bench.py --ablate --phases fwd --rounds 2 --only "enc" > $O/ablate.jsonl 2>&1 || { tail -5 $O/ablate.jsonl; exit 1; }
grep '^{' $O/ablate.jsonl | python -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); print(r['shape'], {k[:-3]: v for k, v in r.items() if k.endswith('_us')})"
echo "[r3e] tests"
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_model_gpu.py -k "bias_grads or residual" > $O/test.log 2>&1
rc=$?; [ $rc -gt 1 ] && { tail -30 $O/test.log; exit 1; }
grep -E "FAILED|passed|failed|Error" $O/test.log | tail -8
run() {  # tag, [VAR=value ...] bench args...
  local tag=$1; shift
  local envs=()
  while [[ "$1" == *=* ]]; do envs+=("$1"); shift; done
  echo "[r3e] $tag ${envs[*]}"
  env "${envs[@]}" timeout -k 10 400 python -u bench.py "$@" > $O/$tag.log 2>&1 || { echo "[r3e] $tag failed rc=$?"; tail -8 $O/$tag.log; return 1; }
  echo "$tag $(grep -h '"metric"' $O/$tag.log | tail -1 | cut -c100-200)"
}
for i in 1 2; do
  run lmchunk_$i DLLM_LMHEAD_FULL_MB=0 --steps 10 --warmup 3 || exit 1
  run lmfull_$i DLLM_LMHEAD_FULL_MB=-1 --steps 10 --warmup 3 || exit 1
done
for i in 1 2; do
  run bartl_b32_colsum_$i DLLM_NORM_BIAS_COLSUM=1 --model bart-large --batch-per-gpu 32 --steps 10 --warmup 3 || exit 1
  run bartl_b32_nocolsum_$i DLLM_NORM_BIAS_COLSUM=0 --model bart-large --batch-per-gpu 32 --steps 10 --warmup 3 || exit 1
done
run t5b_b32 --batch-per-gpu 32 --steps 10 --warmup 3 &&
run t5b_b64 --batch-per-gpu 64 --steps 10 --warmup 3 &&
run t5b_b128 --batch-per-gpu 128 --steps 10 --warmup 3 &&
run bartl_b256 --model bart-large --batch-per-gpu 256 --steps 6 --warmup 2 &&
run t5l_b32 --model t5-large --batch-per-gpu 32 --steps 6 --warmup 2 &&
run flanxl_b16 --model flan-t5-xl --batch-per-gpu 16 --steps 5 --warmup 2 || true
echo "[r3e] profile b8 (graph)"
d=$O/prof8
mkdir -p $d
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d -o run -- python bench.py --batch-per-gpu 8 --steps 20 --warmup 3 --graph off > $O/prof8.log 2>&1 || { tail -5 $O/prof8.log; exit 1; }
db=$(find $d -name "*.db" | head -n 1); csv=$(find $d -name "*kernel_stats.csv" | head -n 1)
python tools/prof_summary.py "${db:-$csv}" 23 > $O/prof8_summary.txt && head -40 $O/prof8_summary.txt
[ -n "$db" ] && rm -f "$db"
exit 0
