#!/bin/bash
# Kernel profiles of the current tree, summarised ON the box (the rocpd databases stay there): t5-base b=256 (bench
# default) and bart-large b=256 (the reference's default model).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/prof2
mkdir -p $O
prof() {  # tag, steps+warmup, bench args...
  local tag=$1 n=$2; shift 2
  local d=/tmp/prof_$tag
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $d -o run -- python bench.py "$@" > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; return 1; }
  python tools/prof_summary.py $(find $d -name "*.db" | head -n 1) $n > $O/${tag}_summary.txt || return 1
  grep -h '"metric"' $O/$tag.log | cut -c1-160
  head -30 $O/${tag}_summary.txt
}
prof t5b256 4 --steps 3 --warmup 1 --graph off || exit 1
prof bartl256 3 --model bart-large --steps 2 --warmup 1 --graph off || exit 1
