#!/bin/bash
# P2P (mailbox) exchange vs RCCL all_gather exchange on one rank: GPU tests of
# the exchange paths, then bench.py --exchange with either mode, interleaved.
#   TAG=name bash tools/p2p_ab.sh [ROUNDS]
set -o pipefail
O=gpurun_out/${TAG:-p2p}; mkdir -p $O
export TMPDIR=/tmp
[ -n "$SKIP_TESTS" ] || timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 \
  --timeout-method thread -k "p2p or two_ranks or exchange" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -1 $O/tests.log
for r in $(seq ${1:-2}); do
  for m in p2p rccl C; do
    if [ $m = C ]; then
      timeout -k 10 200 python bench.py --cpu-seconds 0 --no-second-pass > $O/C$r.json 2> $O/C$r.err || { echo "C failed"; tail -5 $O/C$r.err; exit 1; }
      python3 -c "import json; d=json.loads([l for l in open('$O/C$r.json') if l.startswith('{')][0]); print('C (one GPU, no exchange)', 'step %.2f us' % (d['ms_per_step']*1e3), 'frac', d['roofline']['frac'])"
      continue
    fi
    timeout -k 10 200 python bench.py --exchange --exchange-mode $m --cpu-seconds 0 --no-second-pass > $O/$m$r.json 2> $O/$m$r.err || { echo "$m failed"; tail -5 $O/$m$r.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$O/$m$r.json') if l.startswith('{')][0]); print('$m', 'step %.2f us' % (d['ms_per_step']*1e3), 'kernel %.2f us' % (d['kernel_ms']*1e3), 'p50 %.2f us' % (d['p50_ms']*1e3), 'chain_error', d['chain_error'], 'frac', d['roofline']['frac'])"
  done
done
