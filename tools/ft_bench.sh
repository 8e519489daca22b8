#!/bin/bash
# Full-tree GPU tests, then workloads F and G.   TAG=name bash tools/ft_bench.sh
set -o pipefail
O=gpurun_out/${TAG:-ft}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_fulltree_gpu.py -x -q -m gpu --timeout 120 \
  --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for w in F G; do
  timeout -k 10 200 python bench.py --cpu-seconds 0 --no-second-pass --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || { echo "bench $w failed"; tail -5 $O/bench_$w.err; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/bench_$w.json') if l.startswith('{')][0]); print('$w', d['value'], d['unit'], 'ms/step', d['ms_per_step'], (d.get('roofline') or {}).get('frac'))"
done
