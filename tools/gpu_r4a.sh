#!/bin/bash
# Round 4: graphed data-parallel schedules + entry points on graphs (gpurun -- bash tools/gpu_r4a.sh)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4a
mkdir -p $O
common="--model-ckpt t5-base --synthetic 2560 --max-source-length 1024 --max-target-length 128 --output-dir /tmp/ebench"
timeout -k 10 600 python -u -m pytest tests/test_graph_gpu.py -x -v --timeout 240 --timeout-method thread > $O/graph_tests.log 2>&1 \
  || { tail -40 $O/graph_tests.log; exit 1; }
tail -3 $O/graph_tests.log
DLLM_DIST_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 2 --steps 4 --warmup 2 --batch-per-gpu 16 > $O/gloo2.log 2>&1 \
  || { tail -30 $O/gloo2.log; exit 1; }
grep metric $O/gloo2.log | cut -c1-1500
for g in 1 0; do
  DLLM_GRAPH=$g timeout -k 10 600 python -u train-accelerator.py $common --batch-size 1 --max-steps 80 --max-eval-samples 4 \
    --gen-max-length 8 > $O/acc_b1_g$g.log 2>&1 || { tail -20 $O/acc_b1_g$g.log; exit 1; }
  echo "accelerator b1 graph=$g: $(grep -h train_samples_per_second $O/acc_b1_g$g.log | tail -1)"
done
for g in 1 0; do
  DLLM_GRAPH=$g timeout -k 10 600 python -u train-torchrun.py $common --batch-size 8 --grad-accum 16 --max-steps 6 \
    --evaluation-steps 1000000 --max-eval-samples 8 > $O/torchrun_b8_ga16_g$g.log 2>&1 || { tail -20 $O/torchrun_b8_ga16_g$g.log; exit 1; }
  echo "torchrun b8xGA16 graph=$g: $(grep -h train_runtime $O/torchrun_b8_ga16_g$g.log | tail -1)"
done
DLLM_GRAPH=1 timeout -k 10 600 python -u train-task.py $common --max-steps 60 --max-eval-samples 4 --gen-max-length 8 \
  > $O/task.log 2>&1 || { tail -20 $O/task.log; exit 1; }
tail -4 $O/task.log
