#!/bin/bash
# Per-variant kernel trace of the bench's graph-replayed MPC steps
# (tools/var_<name>.so, VARS): in-step rollout / finalize durations.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/abt
for n in ${VARS:-base}; do
  DIPLOMJOURNEY_MPC_LIB=tools/var_$n.so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv \
    -d gpurun_out/abt/$n -o run -- python3 bench.py --cpu-seconds 0 --no-second-pass \
    > gpurun_out/abt/$n.json 2> gpurun_out/abt/$n.err || exit 1
  python3 tools/step_trace.py gpurun_out/abt/$n/run_kernel_trace.csv $n | tee -a gpurun_out/abt/all.txt || exit 1
done
