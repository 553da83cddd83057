#!/bin/bash
# TunableOp re-tune of the hipBLASLt GEMMs at the bench default (b=256: encoder GEMMs with 262144 rows are not in the
# shipped table), then an interleaved A/B of the merged table vs the old one.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/tune
mkdir -p $O
echo "[tune] tuning run (W4 off: the lib path of every projection)"
DLLM_TUNABLEOP=tune DLLM_TUNABLEOP_DIR=$O PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=40 PYTORCH_TUNABLEOP_VERBOSE=0 \
  timeout -k 10 900 python -u bench.py --steps 2 --warmup 1 --graph off > $O/tune.log 2>&1 || { tail -20 $O/tune.log; exit 1; }
tail -2 $O/tune.log | cut -c1-200
ls -la $O/*.csv
python tools/merge_tunableop.py configs/tunableop/gfx950.csv $O/tunableop_results0.csv -o $O/merged.csv
grep -c "" configs/tunableop/gfx950.csv $O/merged.csv
mkdir -p $O/old && cp configs/tunableop/gfx950.csv $O/old/
for i in 1 2; do
  for t in merged old; do
    if [ $t = merged ]; then cp $O/merged.csv configs/tunableop/gfx950.csv; else cp $O/old/gfx950.csv configs/tunableop/gfx950.csv; fi
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/bench_${t}_$i.log 2>&1 || { tail -5 $O/bench_${t}_$i.log; exit 1; }
    echo "$t $(grep -h '"metric"' $O/bench_${t}_$i.log | tail -1 | cut -c100-190)" | tee -a $O/ab.txt
  done
done
cp $O/old/gfx950.csv configs/tunableop/gfx950.csv
