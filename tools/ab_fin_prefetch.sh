#!/bin/bash
# A/B: the selection with each wave's best controls prefetched during the
# block reduction (in-tree library) vs HEAD~ (tools/var_base.so), chained
# launches; block 0's stage times (tools/var_fin.so, -DMPC_FIN_TRACE); then
# the whole GPU suite on the in-tree library.
set -o pipefail
mkdir -p gpurun_out/s3
O=gpurun_out/s3/ab_prefetch.txt
: > $O
for r in 1 2 3; do
  DIPLOMJOURNEY_MPC_LIB=tools/var_base.so timeout -k 10 120 python tools/time_chain.py >> $O 2>&1 || exit 1
  timeout -k 10 120 python tools/time_chain.py >> $O 2>&1 || exit 1
done
DIPLOMJOURNEY_MPC_LIB=tools/var_fin.so timeout -k 10 120 python tools/probe_chain_block0.py >> $O 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/s3/pytest_prefetch.log 2>&1
rc=$?
grep -v amdgpu.ids $O; tail -2 gpurun_out/s3/pytest_prefetch.log
exit $rc
