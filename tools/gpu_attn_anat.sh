#!/bin/bash
# Attention kernel anatomy: per-feature kernel times (bias / kpm / dropout, saturated vs LUT-path bias) + dK/dV PMC.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/anat
mkdir -p $O
for tag in sat nosat; do
  extra=""; [ $tag = nosat ] && extra="--nosat"
  d=$O/prof_$tag
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $d -o run -- python tools/attn_anat.py --cfg b1k1d1,b0k1d1,b1k1d0,b0k1d0,b1k0d0,b0k0d0 $extra > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; exit 1; }
  db=$(find $d -name "*.db" | head -n 1)
  echo "== $tag"; python tools/prof_summary.py "$db" 1 | grep attn_ | grep "avg" || true
done
echo "== pmc dkdv (b1k1d1)"
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU -d $O/pmc1 -o run -- python tools/attn_anat.py --cfg b1k1d1,b0k0d0 --iters 3 > $O/pmc1.log 2>&1 || { tail -5 $O/pmc1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT -d $O/pmc2 -o run -- python tools/attn_anat.py --cfg b1k1d1,b0k0d0 --iters 3 > $O/pmc2.log 2>&1 || { tail -5 $O/pmc2.log; echo "pmc2 failed"; }
for p in pmc1 pmc2; do
  f=$(find $O/$p -name "*counter_collection.csv" | head -n 1)
  [ -n "$f" ] && python - "$f" <<'EOF'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    if "attn" not in r["Kernel_Name"]: continue
    k = r["Kernel_Name"][:90]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in acc.items():
    print("==", k)
    for c, v in sorted(d.items()): print("   %-24s %16.1f" % (c, v))
EOF
done

# keep only the summaries (the rocpd databases can exceed the copy-back cap)
for p in pmc1 pmc2; do f=$(find $O/$p -name "*.db" | head -n 1); [ -n "$f" ] && python tools/pmc_summary.py $f > $O/${p}_summary.txt; done
find $O -name "*.db" -delete
exit 0
