#!/bin/bash
# Re-measure the non-headline model configs with the current bench.py (one JSON line each) into gpurun_out/configs/.
set -o pipefail
mkdir -p gpurun_out/configs
run() {
  name=$1; shift
  echo "[config_benches] $name: $*"
  timeout -k 10 600 python -u bench.py "$@" > gpurun_out/configs/$name.log 2>&1 || { tail -5 gpurun_out/configs/$name.log; exit 1; }
  tail -1 gpurun_out/configs/$name.log > gpurun_out/configs/$name.json
  cut -c1-160 gpurun_out/configs/$name.json
}
run ours_bart_large_b32 --model bart-large --batch-per-gpu 32 --steps 10 --warmup 3
run ours_bart_large_b256 --model bart-large --batch-per-gpu 256 --steps 5 --warmup 2  # 144 GB peak
run ours_t5_large_b32 --model t5-large --batch-per-gpu 32 --steps 8 --warmup 3
run ours_t5_large_b128 --model t5-large --batch-per-gpu 128 --steps 5 --warmup 2  # 132 GB peak
run ours_flan_t5_xl_b16 --model flan-t5-xl --batch-per-gpu 16 --steps 5 --warmup 2
run ours_t5base_b64_ckpt --model t5-base --batch-per-gpu 64 --grad-ckpt --steps 10 --warmup 3
run ours_flan_xl_long_s4096_b8_ckpt --model flan-t5-xl --batch-per-gpu 8 --src-len 4096 --grad-ckpt --steps 4 --warmup 2
run ours_flan_xl_long_s4096_b8 --model flan-t5-xl --batch-per-gpu 8 --src-len 4096 --steps 4 --warmup 2  # 124 GB peak: no recompute needed on 288 GB
