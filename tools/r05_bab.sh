#!/bin/bash
# Same-box A/B of config B (and C) bench lines: tools/ab_head.so vs the in-tree library,
# interleaved.   TAG=name [WL="B C"] [R=3] bash tools/r05_bab.sh
set -o pipefail
O=gpurun_out/${TAG:-bab5}; mkdir -p $O
for r in $(seq 1 ${R:-3}); do
  for w in ${WL:-B}; do
    for m in head tree; do
      lib=""; [ $m = head ] && lib=$PWD/tools/ab_head.so
      DIPLOMJOURNEY_MPC_LIB=$lib timeout -k 10 200 python bench.py --cpu-seconds 0 --no-second-pass --no-config-d --parity-steps 0 --workload $w $EXTRA > $O/${w}_$m$r.json 2> $O/${w}_$m$r.err || { echo "$m failed"; tail -5 $O/${w}_$m$r.err; exit 1; }
      python3 -c "import json; d=json.loads([l for l in open('$O/${w}_$m$r.json') if l.startswith('{')][0]); print('$w $m', 'step %.2f us' % (d['ms_per_step']*1e3), 'kernel %.2f us' % (d['kernel_ms']*1e3))"
    done
  done
done
