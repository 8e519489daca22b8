#!/bin/bash
# The driver's bench command (--gpus 1 --steps 20 --warmup 5) repeated R times.
#   TAG=name [R=3] bash tools/r05_drv.sh
set -o pipefail
O=gpurun_out/${TAG:-drv}; mkdir -p $O
for r in $(seq 1 ${R:-3}); do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/run$r.json 2> $O/run$r.err || { echo "run $r failed"; tail -5 $O/run$r.err; exit 1; }
  python3 -c "
import json
d = json.loads([l for l in open('$O/run$r.json') if l.startswith('{')][0])
print('run $r', 'step %.2f us' % (d['ms_per_step'] * 1e3), 'kernel %.2f' % (d['kernel_ms'] * 1e3),
      'sustained %.2f' % (d['kernel_ms_sustained'] * 1e3), 'parity', (d.get('parity') or {}).get('identity_rate'))"
done
