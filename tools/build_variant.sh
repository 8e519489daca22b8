#!/bin/bash
# Build one A/B library variant: tools/build_variant.sh NAME [-DFLAG=... ...]
# -> tools/var_NAME.so (select at run time with DIPLOMJOURNEY_MPC_LIB).
set -e
cd "$(dirname "$0")/.."
name=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -Wall \
  -I include "$@" -o tools/var_$name.so diplomjourney_amd/csrc/mpc_rollout.hip
