#!/bin/bash
# Round 4: new-kernel numerics first (fp32 attention, fused LM-head CE, graphs), then the A/B and entry points
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4b
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_attn_f32_gpu.py tests/test_graph_gpu.py "tests/test_grads_gpu.py::test_lm_head_chunked_ce_matches_fp32" \
  tests/test_grads_gpu.py::test_t5_fused_lm_head_matches_materialised_logits tests/test_grads_gpu.py::test_t5_chunked_lm_head_matches_full \
  -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error" $O/tests.log | tail -40
[ $rc -eq 0 ] || exit 1
for f in 1 0; do
  DLLM_LMHEAD_FUSED=$f timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 > $O/bench_fused$f.log 2>&1 || { tail -20 $O/bench_fused$f.log; exit 1; }
  echo "fused=$f $(grep metric $O/bench_fused$f.log | cut -c100-260)"
done
timeout -k 10 600 python -u bench.py --dtype fp32 --batch-per-gpu 16 --steps 6 --warmup 2 > $O/fp32.log 2>&1 || { tail -20 $O/fp32.log; exit 1; }
echo "fp32: $(grep metric $O/fp32.log | cut -c100-260)"
DLLM_DIST_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 2 --steps 4 --warmup 2 --batch-per-gpu 16 > $O/gloo2.log 2>&1 \
  || { tail -30 $O/gloo2.log; exit 1; }
grep metric $O/gloo2.log | cut -c1-1500
common="--model-ckpt t5-base --synthetic 2560 --max-source-length 1024 --max-target-length 128 --output-dir /tmp/ebench"
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
