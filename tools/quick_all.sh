#!/bin/bash
# GPU suite, then config C / B / F bench lines.   TAG=name bash tools/quick_all.sh
set -o pipefail
O=gpurun_out/${TAG:-quick}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for w in C B F; do
  timeout -k 10 200 python bench.py --cpu-seconds 0 --no-second-pass --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || { echo "$w failed"; tail -5 $O/bench_$w.err; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/bench_$w.json') if l.startswith('{')][0]); r=d.get('roofline') or {}; print('$w', '%.4g' % d['value'], d['unit'], 'step %.2f us' % (d['ms_per_step']*1e3), 'kernel', d.get('kernel_ms') or d.get('launch_ms'), 'frac', r.get('frac'), 'valu', (d.get('roofline_valu') or {}).get('frac'))"
done
