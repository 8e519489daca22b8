#!/bin/bash
# In-step traces of the bench per library variant (VARS: tools/var_<name>.so,
# "intree" = the in-tree library) and integrator mode (MODES: rot = two-launch
# rect+rot steps, chain = chained rect+cum steps).  TESTS=1 first runs the
# chained / cumulative-mode GPU tests on the in-tree library.
set -o pipefail
mkdir -p gpurun_out/chain
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_replica.py -x -v --timeout 120 --timeout-method thread -k "chained or cum" > gpurun_out/chain/pytest.log 2>&1 || { tail -30 gpurun_out/chain/pytest.log; exit 1; }
  tail -3 gpurun_out/chain/pytest.log
fi
for rep in $(seq ${REPS:-1}); do
for lib in ${VARS:-intree}; do
for mode in ${MODES:-rot chain}; do
  A="--integrator rect+rot"; [ $mode = chain ] && A="--integrator rect+cum"
  L=""; [ $lib != intree ] && L=tools/var_$lib.so
  tag=$lib-$mode$rep
  DIPLOMJOURNEY_MPC_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/chain/$tag -o run -- python3 bench.py --cpu-seconds 0 --no-second-pass $A > gpurun_out/chain/$tag.json 2> gpurun_out/chain/$tag.err || { tail -5 gpurun_out/chain/$tag.err; exit 1; }
  python3 tools/step_trace.py gpurun_out/chain/$tag/run_kernel_trace.csv $tag || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/chain/$tag.json')); print('$tag', round(d['ms_per_step']*1e3, 2), 'us/step', round(d['kernel_ms']*1e3, 2), 'us kernel')"
done; done; done
