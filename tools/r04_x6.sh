#!/bin/bash
# Exchange-form kernel at 6 waves (tree) vs 5 waves (tools/var_x5.so), serial
# exchange bench interleaved; then a kernel + copy trace of the overlapped
# exchange (where does its step time go?).   TAG=name bash tools/r04_x6.sh
set -o pipefail
O=gpurun_out/${TAG:-x6}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 \
  --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -20 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2 3; do
  for m in w6 w5; do
    lib=""; [ $m = w5 ] && lib=tools/var_x5.so
    DIPLOMJOURNEY_MPC_LIB=$lib timeout -k 10 200 python bench.py --exchange --cpu-seconds 0 --no-second-pass > $O/$m$r.json 2> $O/$m$r.err || { echo "$m failed"; tail -5 $O/$m$r.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$O/$m$r.json') if l.startswith('{')][0]); print('$m', 'step %.2f us' % (d['ms_per_step']*1e3), 'kernel %.2f us' % (d['kernel_ms']*1e3), 'p50 %.2f us' % (d['p50_ms']*1e3), 'frac', d['roofline']['frac'])"
  done
done
timeout -k 10 200 python bench.py --cpu-seconds 0 --no-second-pass > $O/benchC.json 2> $O/benchC.err || { echo "C failed"; tail -5 $O/benchC.err; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$O/benchC.json') if l.startswith('{')][0]); print('C', 'step %.2f us' % (d['ms_per_step']*1e3), 'frac', d['roofline']['frac'])"
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace_ovl -o ovl -- \
  python bench.py --exchange --overlap-exchange --cpu-seconds 0 --no-second-pass --steps 40 --warmup 5 > $O/trace_ovl.log 2>&1 || { echo "trace failed"; tail -5 $O/trace_ovl.log; exit 1; }
echo done
