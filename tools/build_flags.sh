#!/bin/bash
# Build the in-tree sources with extra compiler flags as tools/var_<name>.so
# (developer A/B of compile-time variants; run with tools/with_lib.py).
#   bash tools/build_flags.sh NAME -DMACRO=VALUE ...
set -e
NAME=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ldl -ffp-contract=off \
  -Wall -I include "$@" -o tools/var_$NAME.so diplomjourney_amd/csrc/mpc_rollout.hip
echo tools/var_$NAME.so
