#!/bin/bash
# first GPU probe: device info + HF comparator sweep
set -o pipefail
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/rocm_smi.txt 2>&1 || true
python -c "import torch;print(torch.cuda.get_device_name(0), torch.cuda.get_device_properties(0))" > gpurun_out/devinfo.txt 2>&1
for cfg in "--prec bf16-amp --batch 8" "--prec bf16-amp --batch 16" "--prec bf16-amp --batch 32" "--prec fp32 --batch 16" "--prec bf16 --batch 16" "--prec bf16-amp --batch 16 --attn eager"; do
  timeout -k 10 300 python tools/hf_comparator.py $cfg >> gpurun_out/hf_comparator.jsonl 2>> gpurun_out/hf_comparator.err || { echo "fail $cfg rc=$?"; exit 1; }
  tail -1 gpurun_out/hf_comparator.jsonl
done
