#!/bin/bash
# rocprofv3 --pmc passes (one counter group per run) over the w4 weight-gradient mode vs its NT forward at the same
# FLOPs (tools/gemm_pmc_driver.py 131072 768 2304 wg|w4); summaries in gpurun_out/pmcwg/{wg,w4}.txt
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmcwg; mkdir -p $O
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_WAVES SQ_WAIT_ANY SQ_INSTS_VMEM_WR"
P3="TCC_HIT_sum TCC_MISS_sum"
P4="FETCH_SIZE"
for v in wg w4; do
  n=1
  for P in "$P1" "$P2" "$P3" "$P4"; do
    timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace -d $O/${v}_$n -o run -- python tools/gemm_pmc_driver.py 131072 768 2304 $v > $O/${v}_$n.log 2>&1 || { tail -5 $O/${v}_$n.log; exit 1; }
    n=$((n+1))
  done
  python tools/pmc_summary.py $(find $O/${v}_1 $O/${v}_2 $O/${v}_3 $O/${v}_4 -name "*.db") > $O/${v}.txt || exit 1
done
cat $O/wg.txt $O/w4.txt | grep -v "^== .*Cijk\|rocclr" | head -80
