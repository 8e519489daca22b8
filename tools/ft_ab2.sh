#!/bin/bash
# Round-4 late A/B: tree (fmax-clamped criterion sqrt, per-item leaf index) vs
# tools/var_ftprev.so (commit f2348a8), full-tree launch time under rocprofv3 and
# config-C bench lines; full GPU suite on the tree build first.
set -o pipefail
O=gpurun_out/${TAG:-ftab2}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest ${TESTS:-tests} -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in tree prev tree2 prev2; do
  lib=""; case $v in prev*) lib=tools/var_ftprev.so;; esac
  DIPLOMJOURNEY_MPC_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python bench.py --cpu-seconds 0 --no-second-pass --workload F --steps 30 --warmup 5 > $O/$v.log 2>&1 || { echo "$v failed"; tail -5 $O/$v.log; exit 1; }
  f=$(find $O/$v -name "*kernel_stats.csv" | head -1); python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'k_ft_leaves' in r['Name']: print('$v', r['Name'][:40], r['Calls'], '%.1f us' % (float(r['AverageNs'])/1e3))
"
done
for v in tree prev tree2 prev2; do
  lib=""; case $v in prev*) lib=tools/var_ftprev.so;; esac
  DIPLOMJOURNEY_MPC_LIB=$lib timeout -k 10 120 python bench.py --cpu-seconds 0 --steps 2000 --warmup 200 > $O/C_$v.json 2> $O/C_$v.err || { echo "C $v failed"; tail -5 $O/C_$v.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/C_$v.json').read().strip().splitlines()[-1]); print('C $v', d['ms_per_step']*1e3, 'us', round(d['roofline']['frac'],4))"
done
