#!/bin/bash
# w4 GEMM round: kernel tests, model-level tests, microbench vs hipBLASLt, PMC passes, whole-step A/B (DLLM_W4_GEMM).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/w4c
mkdir -p $O
step() { echo "[w4run] $*"; }
step tests
timeout -k 10 900 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gemm_w4_gpu.py \
  tests/test_model_gpu.py tests/test_graph_gpu.py tests/test_kernels_gpu.py tests/test_grads_gpu.py -s > $O/test.log 2>&1
rc=$?; [ $rc -gt 1 ] && { tail -40 $O/test.log; exit 1; }
grep -E "FAILED|passed|failed" $O/test.log | tail -15
tail -2 $O/test.log
grep -E "^\[parity" $O/test.log | head
step microbench
timeout -k 10 500 python -u tools/gemm_w4_bench.py --rounds 2 > $O/bench.jsonl 2>&1 || { tail -5 $O/bench.jsonl; exit 1; }
for shp in "131072 768 2304 w4" "131072 3072 768 w4"; do
  tag=$(echo $shp | tr ' ' _)
  step pmc $tag
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace -d $O/pmc1_$tag -o run -- python tools/gemm_pmc_driver.py $shp > $O/pmc1_$tag.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM --kernel-trace -d $O/pmc2_$tag -o run -- python tools/gemm_pmc_driver.py $shp > $O/pmc2_$tag.log 2>&1 || exit 1
  python tools/pmc_summary.py $(find $O/pmc1_$tag $O/pmc2_$tag -name "*.db") > $O/pmc_$tag.txt 2>&1
  find $O/pmc1_$tag $O/pmc2_$tag -name "*.db" -delete
done
for v in 0 1 0 1; do
  step bench W4=$v
  DLLM_W4_GEMM=$v timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > $O/bench_w4_$v.log 2>&1 || { tail -5 $O/bench_w4_$v.log; exit 1; }
  tail -1 $O/bench_w4_$v.log | cut -c1-200 | tee -a $O/ab.txt
done
cat $O/bench.jsonl | cut -c1-330
