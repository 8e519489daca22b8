#!/bin/bash
# A/B of chained-kernel work distributions (round 2): tile per block (base),
# equal per-wave runs (even: -DMPC_CHAIN_EVEN=1), dynamic tile claims (claim:
# -DMPC_CHAIN_CLAIM=1, with -DMPC_CHAIN_TIMELINE for tlclaim), each built with
# tools/build_variant.sh; then the claim variant's timeline and chain tests.
# The even / claim code paths were removed after this A/B (both slower); they
# are in commit 48e9dbb.
set -o pipefail
mkdir -p gpurun_out/s3
O=gpurun_out/s3/ab_claim.txt
: > $O
for r in 1 2; do
  for var in ${VARS:-base xclaim}; do
    DIPLOMJOURNEY_MPC_LIB=tools/var_$var.so timeout -k 10 120 python tools/time_chain.py >> $O 2>&1 || exit 1
  done
done
DIPLOMJOURNEY_MPC_LIB=tools/var_tl${TLV:-xclaim}.so timeout -k 10 120 python tools/chain_timeline.py > gpurun_out/s3/timeline_claim.txt 2>&1 || exit 1
DIPLOMJOURNEY_MPC_LIB=tools/var_${TV:-xclaim}.so timeout -k 10 400 python -u -m pytest tests -x -q -m gpu -k "chain or short_and_long" --timeout 120 --timeout-method thread > gpurun_out/s3/pytest_claim.log 2>&1
rc=$?
grep "chained launch" $O; tail -3 gpurun_out/s3/pytest_claim.log; head -16 gpurun_out/s3/timeline_claim.txt
exit $rc
