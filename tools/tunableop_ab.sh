#!/bin/bash
# Interleaved A/B of the in-tree TunableOp table (new) against tools/ab_tune_old.csv (old) on the default bench.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/tune_ab
mkdir -p $O
cp configs/tunableop/gfx950.csv $O/new.csv
for i in 1 2 3; do
  for t in new old; do
    if [ $t = new ]; then cp $O/new.csv configs/tunableop/gfx950.csv; else cp tools/ab_tune_old.csv configs/tunableop/gfx950.csv; fi
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 "$@" > $O/bench_${t}_$i.log 2>&1 || { tail -5 $O/bench_${t}_$i.log; exit 1; }
    echo "$t $(grep -h '"metric"' $O/bench_${t}_$i.log | tail -1 | cut -c100-190)" | tee -a $O/ab.txt
  done
done
cp $O/new.csv configs/tunableop/gfx950.csv
