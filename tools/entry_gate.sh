#!/bin/bash
# Entry-point half of the regression gate: the reference's own micro-batch loops through the
# three entry points, run in the round-start tree (GATE_BASE, built under ab/) and the current tree, interleaved, REPS
# rounds; one line per run with the steady samples/s (after the warm-up / capture steps) in gpurun_out/<tag>/entry.txt.
#
#   gpurun --timeout 1200 -- bash tools/entry_gate.sh entry [REPS]
set -o pipefail
TAG=${1:-entry}
REPS=${2:-2}
BASE=${GATE_BASE:-ab/r6base}
O=gpurun_out/$TAG
mkdir -p $O
common="--model-ckpt t5-base --synthetic 4096 --max-source-length 1024 --max-target-length 128 --output-dir /tmp/egate"
declare -A CMDS
CMDS[accelerator_b1]="train-accelerator.py $common --batch-size 1 --max-steps 200 --max-eval-samples 8 --gen-max-length 16"
CMDS[torchrun_b1_ga16]="train-torchrun.py $common --batch-size 1 --grad-accum 16 --max-steps 24 --evaluation-steps 1000000 --max-eval-samples 8"
CMDS[torchrun_b8_ga16]="train-torchrun.py $common --batch-size 8 --grad-accum 16 --max-steps 16 --evaluation-steps 1000000 --max-eval-samples 8"
for rep in $(seq 1 $REPS); do
  for name in accelerator_b1 torchrun_b1_ga16 torchrun_b8_ga16; do
    for arm in base cur; do
      dir=.; [ $arm = base ] && dir=$BASE
      log=$O/${name}_${arm}_${rep}.log
      (cd $dir && timeout -k 10 600 python ${CMDS[$name]}) > $log 2>&1 || { echo "FAILED $name $arm"; tail -20 $log; exit 1; }
      v=$(grep -ho '"train_steady_samples_per_second": [0-9.]*' $log | tail -1 | awk '{print $2}')
      echo "$name $arm rep$rep steady_samples_per_s $v" | tee -a $O/entry.txt
    done
  done
done
python - "$O/entry.txt" <<'EOF'
import collections, statistics, sys
v = collections.defaultdict(list)
for line in open(sys.argv[1]):
    p = line.split()
    if len(p) == 5 and p[4] not in ("", "None"):
        v[(p[0], p[1])].append(float(p[4]))
for name in sorted({k[0] for k in v}):
    b, c = statistics.median(v[(name, "base")]), statistics.median(v[(name, "cur")])
    print(f"{name:20s} base {b:9.2f}  cur {c:9.2f}  {100 * (c / b - 1):+6.2f} %")
EOF
