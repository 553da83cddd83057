#!/bin/bash
# PMC passes on the fused GEMM vs hipBLASLt (same shape): wave-state split, MFMA busy, LDS conflicts, L2 hits.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc36
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/pmc36/p1 -o p1 -- python $GRAFT_REPO_ROOT/tools/gemm_pmc_driver.py > $GRAFT_REPO_ROOT/gpurun_out/pmc36/p1.log 2>&1 || { echo P1_FAIL; tail -5 $GRAFT_REPO_ROOT/gpurun_out/pmc36/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVES --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/pmc36/p2 -o p2 -- python $GRAFT_REPO_ROOT/tools/gemm_pmc_driver.py > $GRAFT_REPO_ROOT/gpurun_out/pmc36/p2.log 2>&1 || { echo P2_FAIL; tail -5 $GRAFT_REPO_ROOT/gpurun_out/pmc36/p2.log; exit 1; }
ls -R $GRAFT_REPO_ROOT/gpurun_out/pmc36 | head -20
