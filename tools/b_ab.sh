#!/bin/bash
# Config B: small-horizon chained path (tree) vs tools/var_nosmall.so, interleaved; timeline.
set -o pipefail
O=gpurun_out/${TAG:-bab}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k "chain" > $O/tests.log 2>&1 || { echo "tests failed"; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do
  for m in small nosmall; do
    lib=""; [ $m = nosmall ] && lib=tools/var_nosmall.so
    DIPLOMJOURNEY_MPC_LIB=$lib timeout -k 10 200 python bench.py --cpu-seconds 0 --no-second-pass --workload B > $O/$m$r.json 2> $O/$m$r.err || { echo "$m failed"; tail -5 $O/$m$r.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$O/$m$r.json') if l.startswith('{')][0]); print('$m', 'step %.2f us' % (d['ms_per_step']*1e3), 'kernel %.2f us' % (d['kernel_ms']*1e3))"
  done
done
timeout -k 10 150 python tools/chain_timeline.py run 100000 3 > $O/timeline_B.txt 2>&1 || { echo "timeline failed"; exit 1; }
grep -v "^JSON" $O/timeline_B.txt | tail -4
