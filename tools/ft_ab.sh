#!/bin/bash
# Full-tree leaf kernel A/B: tree vs tools/var_ft0.so (round-start) vs tools/var_ftcmp.so,
# kernel stats under rocprofv3 of workload F; full-tree tests on the tree build first.
set -o pipefail
O=gpurun_out/${TAG:-ftab}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_fulltree_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in tree ftcmp ftu2 tree2; do
  lib=""; [ $v = ftu2 ] && lib=tools/var_ftu2.so; [ $v = ftcmp ] && lib=tools/var_ftcmp.so
  DIPLOMJOURNEY_MPC_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python bench.py --cpu-seconds 0 --no-second-pass --workload F --steps 30 --warmup 5 > $O/$v.log 2>&1 || { echo "$v failed"; tail -5 $O/$v.log; exit 1; }
  f=$(find $O/$v -name "*kernel_stats.csv" | head -1); python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'k_ft_leaves' in r['Name']: print('$v', r['Name'][:40], r['Calls'], '%.1f us' % (float(r['AverageNs'])/1e3))
"
done
