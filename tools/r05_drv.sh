#!/bin/bash
# The driver's bench command (--gpus 1 --steps 20 --warmup 5) repeated, with and
# without the CPU baseline leg before it.   TAG=name [R=3] bash tools/r05_drv.sh
set -o pipefail
O=gpurun_out/${TAG:-drv}; mkdir -p $O
for r in $(seq 1 ${R:-3}); do
  for m in cpu nocpu; do
    extra=""; [ $m = nocpu ] && extra="--cpu-seconds 0"
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 $extra > $O/$m$r.json 2> $O/$m$r.err || { echo "$m failed"; tail -5 $O/$m$r.err; exit 1; }
    python3 -c "
import json, re
d = json.loads([l for l in open('$O/$m$r.json') if l.startswith('{')][0])
print('$m', 'step %.2f us' % (d['ms_per_step'] * 1e3), 'kernel %.2f' % (d['kernel_ms'] * 1e3), 'sustained %.2f' % (d['kernel_ms_sustained'] * 1e3))"
  done
done
