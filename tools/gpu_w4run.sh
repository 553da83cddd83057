set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/w4b
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_w4_gpu.py > gpurun_out/w4b/test.log 2>&1 || { tail -30 gpurun_out/w4b/test.log; exit 1; }
tail -2 gpurun_out/w4b/test.log
timeout -k 10 500 python -u tools/gemm_w4_bench.py --rounds 2 > gpurun_out/w4b/bench.jsonl 2>&1 || { tail -5 gpurun_out/w4b/bench.jsonl; exit 1; }
for shp in "131072 768 2304 w4" "131072 3072 768 w4"; do
  tag=$(echo $shp | tr ' ' _)
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace -d gpurun_out/w4b/pmc1_$tag -o run -- python tools/gemm_pmc_driver.py $shp > gpurun_out/w4b/pmc1_$tag.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM --kernel-trace -d gpurun_out/w4b/pmc2_$tag -o run -- python tools/gemm_pmc_driver.py $shp > gpurun_out/w4b/pmc2_$tag.log 2>&1 || exit 1
  python tools/pmc_summary.py $(find gpurun_out/w4b/pmc1_$tag gpurun_out/w4b/pmc2_$tag -name "*.db") > gpurun_out/w4b/pmc_$tag.txt 2>&1
  find gpurun_out/w4b/pmc1_$tag gpurun_out/w4b/pmc2_$tag -name "*.db" -delete
done
cat gpurun_out/w4b/bench.jsonl
