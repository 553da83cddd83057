set -e
cd /root/repo
# the base tree's tools/ is not uploaded (.gpurunignore): run this tree's bench file against the base package
mkdir -p ab/r4base/tools && cp tools/attn_bench.py ab/r4base/tools/
for t in old new; do
  if [ $t = old ]; then R=ab/r4base; else R=.; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/aq_$t -o run -- python $R/tools/attn_bench.py --quick > gpurun_out/aq_$t.log 2>&1
done
for t in old new; do echo "== $t"; find gpurun_out/aq_$t -name "*kernel_stats.csv" | head -1 | xargs -I{} python -c "
import csv,sys
for r in csv.DictReader(open('{}')):
    if 'attn' in r['Name']: print(r['Name'][:90], r['Calls'], r['AverageNs'])
"; done
