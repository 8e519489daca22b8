#!/bin/bash
# Interleaved kernel-only A/B of tools/var_<name>.so (VARS), REPS rounds;
# STEP=1 adds the bench's MPC step time per variant.
set -o pipefail
mkdir -p gpurun_out/abk
for rep in $(seq ${REPS:-2}); do
for n in ${VARS:-base}; do
  DIPLOMJOURNEY_MPC_LIB=tools/var_$n.so timeout -k 10 120 python tools/ab_kernel.py ${ARGS:-} 2> gpurun_out/abk/$n.err | tee -a gpurun_out/abk/all.jsonl || exit 1
  if [ -n "${STEP:-}" ]; then   # also the bench's MPC step (rollout + finalize, graph-replayed)
    DIPLOMJOURNEY_MPC_LIB=tools/var_$n.so timeout -k 10 120 python bench.py --cpu-seconds 0 --no-second-pass 2> gpurun_out/abk/$n.bench.err | \
      python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'lib': '$n', 'ms_per_step': d['ms_per_step'], 'kernel_ms': d['kernel_ms'], 'p50_ms': d['p50_ms']}))" | tee -a gpurun_out/abk/all.jsonl || exit 1
  fi
done; done
