#!/bin/bash
# rocprofv3 --pmc passes (one counter group per run) over the w4 NT forward and hipBLASLt's kernel on the same shape
# (tools/gemm_pmc_driver.py M K N w4 runs both); summaries in gpurun_out/pmcnt/<shape>.txt
#   bash tools/pmc_w4_lib.sh "524288 768 2304" "524288 3072 768"
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmcnt; mkdir -p $O
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_WAVES SQ_WAIT_ANY SQ_INSTS_VMEM_WR"
P3="TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum"
P4="FETCH_SIZE"
P5="WRITE_SIZE TCC_EA0_RDREQ_sum"
for shape in "$@"; do
  tag=$(echo $shape | tr ' ' x)
  n=1
  for P in "$P1" "$P2" "$P3" "$P4" "$P5"; do
    timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace -d $O/${tag}_$n -o run -- python tools/gemm_pmc_driver.py $shape w4 > $O/${tag}_$n.log 2>&1 || { tail -5 $O/${tag}_$n.log; exit 1; }
    n=$((n+1))
  done
  python tools/pmc_summary.py $(find $O/${tag}_1 $O/${tag}_2 $O/${tag}_3 $O/${tag}_4 $O/${tag}_5 -name "*.db") > $O/${tag}.txt || exit 1
  echo "### $shape"; cat $O/${tag}.txt
done
