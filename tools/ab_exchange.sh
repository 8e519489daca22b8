#!/bin/bash
# Same-box A/B of the exchange step (bench.py --exchange: 1-rank RCCL group,
# graph-captured) for the in-tree library and tools/var_$1.so, ROUNDS rounds.
#   TAG=name bash tools/ab_exchange.sh VARIANT [ROUNDS]
set -o pipefail
O=gpurun_out/${TAG:-abx}; mkdir -p $O
for r in $(seq ${2:-2}); do
  for lib in - tools/var_$1.so; do
    if [ "$lib" = - ]; then unset DIPLOMJOURNEY_MPC_LIB; else export DIPLOMJOURNEY_MPC_LIB=$PWD/$lib; fi
    timeout -k 10 200 python bench.py --exchange --cpu-seconds 0 --no-second-pass > $O/x.out 2> $O/x.err || { echo "$lib failed"; tail -3 $O/x.err; exit 1; }
    grep '^{' $O/x.out | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('$lib', 'exchange step %.2f us' % (d['ms_per_step']*1e3))"
  done
done
unset DIPLOMJOURNEY_MPC_LIB
