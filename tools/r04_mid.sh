#!/bin/bash
# Mid-round check: GPU suite, config B (bench + timeline), full tree (F/G + kernel stats).
set -o pipefail
O=gpurun_out/${TAG:-mid}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
  > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  timeout -k 10 200 python bench.py --cpu-seconds 0 --no-second-pass --workload B > $O/bench_B$r.json 2> $O/bench_B$r.err || { echo "B failed"; tail -5 $O/bench_B$r.err; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/bench_B$r.json') if l.startswith('{')][0]); print('B', 'step %.2f us' % (d['ms_per_step']*1e3), 'kernel %.2f us' % (d['kernel_ms']*1e3), 'p50_host', d.get('p50_host_ms'))"
done
timeout -k 10 150 python tools/chain_timeline.py run 100000 3 > $O/timeline_B.txt 2>&1 || { echo "timeline failed"; tail -5 $O/timeline_B.txt; exit 1; }
grep -v "^JSON" $O/timeline_B.txt | tail -4
TAG=$TAG/ft bash tools/ft_bench.sh && TAG=$TAG/ftprof bash tools/ft_prof.sh
