#!/bin/bash
# The exchange step on one rank (1-rank RCCL group, graph-captured), serial
# (launch -> all_gather -> launch) vs overlapped (--overlap-exchange: the
# all_gather beside the next launch, CU-masked launch stream), interleaved
# ROUNDS times; then the PMC traffic passes of the exchange-form kernel.
#   TAG=name bash tools/xchg_ab.sh [ROUNDS]
set -o pipefail
O=gpurun_out/${TAG:-xchg}; mkdir -p $O
export TMPDIR=/tmp
for r in $(seq ${1:-2}); do
  for m in serial overlap; do
    a=""; [ $m = overlap ] && a="--overlap-exchange"
    timeout -k 10 200 python bench.py --exchange --cpu-seconds 0 --no-second-pass $a > $O/$m$r.json 2> $O/$m$r.err || { echo "$m failed"; tail -5 $O/$m$r.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$O/$m$r.json') if l.startswith('{')][0]); print('$m', 'step %.2f us' % (d['ms_per_step']*1e3), 'kernel %.2f us' % (d['kernel_ms']*1e3), 'p50 %.2f us' % (d['p50_ms']*1e3), 'chain_error', d['chain_error'], d['config']['launch'])"
  done
done
