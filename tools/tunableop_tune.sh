#!/bin/bash
# TunableOp re-tune of the hipBLASLt GEMMs at the bench default (b=512 since late round 3: encoder GEMMs with 524288 rows
# and the full-logits LM head are not in the shipped table).  Writes gpurun_out/tune/merged.csv; the A/B against the
# previous table is tools/tunableop_ab.sh.  A heartbeat line every 50 s keeps the (otherwise silent) tuning run alive.
set -o pipefail
export TMPDIR=/tmp
O=${TUNE_OUT:-gpurun_out/tune}
mkdir -p $O
( while sleep 50; do echo "[tune] alive: $(grep -vc '^Validator' $O/tunableop_results0.csv 2>/dev/null) solutions"; done ) &
HB=$!
trap "kill $HB" EXIT
echo "[tune] tuning run"
DLLM_TUNABLEOP=tune:$O PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=${TUNE_MS:-40} PYTORCH_TUNABLEOP_VERBOSE=0 \
  timeout -k 10 ${TUNE_TIMEOUT:-1000} python -u bench.py --steps 1 --warmup 1 --graph off "$@" > $O/tune.log 2>&1 || { tail -20 $O/tune.log; exit 1; }
tail -2 $O/tune.log | cut -c1-200
python tools/merge_tunableop.py configs/tunableop/gfx950.csv $O/tunableop_results0.csv -o $O/merged.csv
grep -c "" configs/tunableop/gfx950.csv $O/merged.csv
