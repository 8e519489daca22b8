#!/bin/bash
# Build the HIP library of a git revision (or a source dir) as tools/var_<name>.so
# for same-box A/B runs (tools/ab_chain.py).   bash tools/build_variant.sh NAME REV
set -e
NAME=$1; REV=$2
D=$(mktemp -d)
git archive "$REV" diplomjourney_amd/csrc include | tar -x -C "$D"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ldl -ffp-contract=off \
  -I "$D/include" -o tools/var_$NAME.so "$D/diplomjourney_amd/csrc/mpc_rollout.hip"
rm -rf "$D"
echo tools/var_$NAME.so
