#!/bin/bash
# Interleaved kernel-only A/B of tools/var_<name>.so (VARS), REPS rounds.
set -o pipefail
mkdir -p gpurun_out/abk
for rep in $(seq ${REPS:-2}); do
for n in ${VARS:-base}; do
  DIPLOMJOURNEY_MPC_LIB=tools/var_$n.so timeout -k 10 120 python tools/ab_kernel.py ${ARGS:-} 2> gpurun_out/abk/$n.err | tee -a gpurun_out/abk/all.jsonl || exit 1
done; done
