#!/bin/bash
# rocprofv3 kernel stats of workload F: the tree's library vs tools/var_noprune.so
set -o pipefail
O=gpurun_out/${TAG:-ftprof}; mkdir -p $O
export TMPDIR=/tmp
for v in tree noprune; do
  lib=""; [ $v = noprune ] && lib=tools/var_noprune.so
  DIPLOMJOURNEY_MPC_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python bench.py --cpu-seconds 0 --no-second-pass --workload F --steps 30 --warmup 5 > $O/$v.log 2>&1 || { echo "$v failed"; tail -5 $O/$v.log; exit 1; }
  echo "== $v"; f=$(find $O/$v -name "*kernel_stats.csv" | head -1); python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    print(r['Name'][:60], r['Calls'], r['AverageNs'])
"
done
