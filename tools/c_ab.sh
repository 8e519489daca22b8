#!/bin/bash
# Config C A/B: tree vs tools/var_prev.so, interleaved; then VALU PMC passes.
set -o pipefail
O=gpurun_out/${TAG:-cab}; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  for m in tree prev; do
    lib=""; [ $m = prev ] && lib=tools/var_prev.so
    DIPLOMJOURNEY_MPC_LIB=$lib timeout -k 10 200 python bench.py --cpu-seconds 0 --no-second-pass > $O/$m$r.json 2> $O/$m$r.err || { echo "$m failed"; tail -5 $O/$m$r.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$O/$m$r.json') if l.startswith('{')][0]); print('$m', 'step %.2f us' % (d['ms_per_step']*1e3), 'kernel %.2f us' % (d['kernel_ms']*1e3), 'frac', d['roofline']['frac'])"
  done
done
TAG=$TAG/valu bash tools/pmc_valu.sh > $O/valu.log 2>&1 && tail -4 $O/valu.log
