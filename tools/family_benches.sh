#!/bin/bash
# One bench.py line per supported model family at its round-4 reference configuration, current tree:
# every family still trains on the current routing (ReLU FFNs of Pegasus / M2M100 / NLLB on the w4 epilogue, the
# row-Weyl FFN dropout in every activation path).  Summary: gpurun_out/<tag>/families.txt
set -o pipefail
TAG=${1:-families}
O=gpurun_out/$TAG; mkdir -p $O
run() {
  name=$1; shift
  timeout -k 10 420 python -u bench.py "$@" > $O/$name.log 2>&1 || { echo "FAILED $name"; tail -5 $O/$name.log; exit 1; }
  python - "$name" "$O/$name.log" <<'PY' | tee -a $O/families.txt
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"{sys.argv[1]:28s} b={d['config']['per_gpu_batch']:<4d} {d['value']:9.2f} samples/s {d['ms_per_step']:8.1f} ms/step  "
      f"MFU {d.get('mfu', float('nan')):.3f}")
PY
}
run t5-base-b128 --model t5-base --batch-per-gpu 128 --steps 8 --warmup 3
run flan-t5-base-b128 --model flan-t5-base --batch-per-gpu 128 --steps 8 --warmup 3
run flan-t5-large-b32 --model flan-t5-large --batch-per-gpu 32 --steps 6 --warmup 2
run mt5-base-b128 --model mt5-base --batch-per-gpu 128 --steps 6 --warmup 2
run umt5-base-b128 --model umt5-base --batch-per-gpu 128 --steps 6 --warmup 2
run mbart-large-cc25-b128 --model mbart-large-cc25 --batch-per-gpu 128 --steps 6 --warmup 2
run pegasus-large-b128 --model pegasus-large --batch-per-gpu 128 --steps 6 --warmup 2
run nllb-200-distilled-600m-b128 --model nllb-200-distilled-600m --batch-per-gpu 128 --steps 6 --warmup 2
run opus-mt-en-de-b256 --model opus-mt-en-de --batch-per-gpu 256 --src-len 512 --steps 8 --warmup 3
run plbart-base-b128 --model plbart-base --batch-per-gpu 128 --steps 8 --warmup 3
run blenderbot-400m-b64 --model blenderbot-400m-distill --batch-per-gpu 64 --src-len 128 --tgt-len 128 --steps 8 --warmup 3
