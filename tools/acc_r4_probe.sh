#!/bin/bash
# train-accelerator.py at the reference's micro-batch (b=1, one optimizer step per sample): round-4-end tree (ab/r4end,
# built with its own library) vs the current tree, interleaved; steady samples/s per run in gpurun_out/acc_r4/acc.txt.
# PROF=1: one rocprofv3 --kernel-trace --stats run of each (kernel_stats.csv per arm) instead.
set -o pipefail
O=gpurun_out/acc_r4
mkdir -p $O
common="--model-ckpt t5-base --synthetic 4096 --max-source-length 1024 --max-target-length 128 --output-dir /tmp/egate --batch-size 1 --max-evaluation-samples 8 --gen-max-length 16"
common="${common/--max-evaluation-samples/--max-eval-samples}"
if [ "${PROF:-0}" = 1 ]; then
  for arm in r4 cur; do
    dir=$PWD; [ $arm = r4 ] && dir=$PWD/ab/r4end
    (cd $dir && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OLDPWD/$O/prof_$arm -o run -- python train-accelerator.py $common --max-steps 60) > $O/prof_${arm}.log 2>&1 || { echo FAILED $arm; tail -20 $O/prof_${arm}.log; exit 1; }
    find $O/prof_$arm -type f ! -name "*stats*" -delete
    echo "profiled $arm"
  done
  exit 0
fi
# ARMS: r4 (round-4-end tree), cur (this tree), and cur_<name> arms with DLLM_ROUTE=<ROUTE_<name>> (e.g. ARMS="r4 cur
# cur_ffn" ROUTE_ffn=ffn_min_rows=0)
for rep in 1 2; do
  for arm in ${ARMS:-r4 cur}; do
    dir=.; [ $arm = r4 ] && dir=ab/r4end
    rv=ROUTE_${arm#cur_}; route=""; [ "${arm#cur_}" != "$arm" ] && route=${!rv}
    (cd $dir && DLLM_ROUTE=$route timeout -k 10 300 python train-accelerator.py $common --max-steps 200) > $O/${arm}_${rep}.log 2>&1 || { echo FAILED $arm; tail -20 $O/${arm}_${rep}.log; exit 1; }
    v=$(grep -ho '"train_steady_samples_per_second": [0-9.]*' $O/${arm}_${rep}.log | tail -1)
    echo "$arm rep$rep $v" | tee -a $O/acc.txt
  done
done
