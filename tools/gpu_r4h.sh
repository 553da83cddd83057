#!/bin/bash
# Round 4: dK/dV kernel timing ablations (csrc/attn.hip DKDV_ABLATE builds in ab_so/), T5 encoder shape B=32;
# args: variant names (ab_so/<name>.so); PMC=1 adds a bank-conflict / issue counter pass on the default build
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4h
mkdir -p $O
so=$(ls distributed_llms_example_amd/_C*.so | head -n 1)
cp "$so" /tmp/_C_current.so
for round in 1 2; do
  for v in "$@"; do
    cp ab_so/$v.so "$so"
    timeout -k 10 300 python tools/attn_bench.py --quick > $O/${v}_$round.log 2>&1 || { cp /tmp/_C_current.so "$so"; tail -5 $O/${v}_$round.log; exit 1; }
    echo "$v: $(python -c "import json,sys; [print(round(json.loads(l)['bwd_ms'],4), round(json.loads(l)['fwd_ms'],4), end=' ') for l in open('$O/${v}_$round.log') if l.startswith('{')]")"
  done
done
cp /tmp/_C_current.so "$so"
if [ "${PMC:-0}" = 1 ]; then
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT -d $O/pmc2 -o run -- python tools/attn_anat.py --cfg b1k1d1 --iters 3 > $O/pmc2.log 2>&1 || { tail -5 $O/pmc2.log; exit 1; }
  f=$(find $O/pmc2 -name "*.db" | head -n 1); python tools/pmc_summary.py $f > $O/pmc2_summary.txt && cat $O/pmc2_summary.txt | grep -A9 "attn_"
  find $O/pmc2 -name "*.db" -delete
fi
