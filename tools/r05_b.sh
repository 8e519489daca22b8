#!/bin/bash
# Config B's block-0 chain after the early publication: chained-episode GPU
# tests, the B and C bench lines, the B timeline.   TAG=name bash tools/r05_b.sh
set -o pipefail
O=gpurun_out/${TAG:-b5}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k "chain or episode or tiled" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for w in B C; do
  timeout -k 10 300 python bench.py --cpu-seconds 0 --no-second-pass --no-config-d --parity-steps 0 --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || { echo "bench $w failed"; tail -5 $O/bench_$w.err; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/bench_$w.json') if l.startswith('{')][0]); print('$w', 'step %.2f us' % (d['ms_per_step']*1e3), 'kernel %.2f us' % (d['kernel_ms']*1e3), 'frac', d['roofline']['frac'])"
done
timeout -k 10 150 python tools/chain_timeline.py run 100000 3 > $O/timeline_B.txt 2>&1 || { echo "timeline failed"; tail -5 $O/timeline_B.txt; exit 1; }
grep -v "^JSON" $O/timeline_B.txt | tail -4
