#!/bin/bash
# PMC passes on the attention kernels (t5-base encoder shape, bias + padding + dropout).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc39
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/pmc39/p1 -o p1 -- python $GRAFT_REPO_ROOT/tools/attn_bench.py --quick > $GRAFT_REPO_ROOT/gpurun_out/pmc39/p1.log 2>&1 || { echo P1_FAIL; tail -5 $GRAFT_REPO_ROOT/gpurun_out/pmc39/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/pmc39/p2 -o p2 -- python $GRAFT_REPO_ROOT/tools/attn_bench.py --quick > $GRAFT_REPO_ROOT/gpurun_out/pmc39/p2.log 2>&1 || { echo P2_FAIL; tail -5 $GRAFT_REPO_ROOT/gpurun_out/pmc39/p2.log; exit 1; }
echo done
