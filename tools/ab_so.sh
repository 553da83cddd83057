#!/bin/bash
# A/B two builds of the native extension on one box: swap the in-tree _C .so between runs of one command.
#   bash tools/ab_so.sh TAG A.so B.so ROUNDS CMD...      (prints the last output line of every run)
set -o pipefail
tag=$1; a=$2; b=$3; rounds=$4; shift 4
so=$(ls distributed_llms_example_amd/_C*.so | head -n 1)
cp "$so" /tmp/_C_current.so
mkdir -p gpurun_out/$tag
rc=0
for i in $(seq 1 "$rounds"); do
  for side in A B; do
    f=$a; [ $side = B ] && f=$b
    cp "$f" "$so"
    timeout -k 10 300 "$@" > gpurun_out/$tag/${side}_$i.log 2>&1 || { rc=$?; tail -5 gpurun_out/$tag/${side}_$i.log; break 2; }
    tail -n "${AB_TAIL:-1}" gpurun_out/$tag/${side}_$i.log | sed "s/^/$side /"
  done
done
cp /tmp/_C_current.so "$so"
exit $rc
