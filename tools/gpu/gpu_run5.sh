#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/attn_bench.py > gpurun_out/attn_bench.jsonl 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/attn_bench.jsonl; exit 1; }
cat gpurun_out/attn_bench.jsonl
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT -d $GRAFT_REPO_ROOT/gpurun_out/pmc1 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/attn_bench.py --quick > $GRAFT_REPO_ROOT/gpurun_out/pmc1.log 2>&1 || { echo PMC_FAIL; tail -20 $GRAFT_REPO_ROOT/gpurun_out/pmc1.log; exit 1; }
echo PMC_OK
