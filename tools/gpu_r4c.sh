#!/bin/bash
# Round 4: per-shape kernel trace of the t5-base b=512 step and of the fp32 b=16 step (gpurun -- bash tools/gpu_r4c.sh)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4c
mkdir -p $O
for cfg in "b512:--steps 2 --warmup 1 --graph off" "fp32:--dtype fp32 --batch-per-gpu 16 --steps 2 --warmup 1 --graph off"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  d=$O/prof_$tag
  mkdir -p $d
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $d -o run -- python bench.py $args > $O/prof_$tag.log 2>&1 || { tail -20 $O/prof_$tag.log; exit 1; }
  db=$(find $d -name "*.db" | head -n 1)
  csv=$(find $d -name "*kernel_stats.csv" | head -n 1)
  python tools/prof_summary.py "${db:-$csv}" 3 > $O/summary_$tag.txt && head -24 $O/summary_$tag.txt
  tcsv=$(find $d -name "*kernel_trace.csv" | head -n 1)
  python tools/trace_shapes.py "${db:-$tcsv}" 3 60 > $O/shapes_$tag.txt && head -40 $O/shapes_$tag.txt
  rm -f $d/*/*.db 2>/dev/null; find $d -name "*.db" -size +50M -delete
done
common="--model-ckpt t5-base --synthetic 4096 --max-source-length 1024 --max-target-length 128 --output-dir /tmp/ebench"
for g in 1 0; do
  DLLM_GRAPH=$g timeout -k 10 600 python -u train-torchrun.py $common --batch-size 8 --grad-accum 16 --max-steps 16 \
    --evaluation-steps 1000000 --max-eval-samples 8 > $O/torchrun_b8_ga16_g$g.log 2>&1 || { tail -20 $O/torchrun_b8_ga16_g$g.log; exit 1; }
  echo "torchrun b8xGA16 graph=$g: $(grep -h train_runtime $O/torchrun_b8_ga16_g$g.log | tail -1)"
done
