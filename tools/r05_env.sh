#!/bin/bash
# Graph-replay submission probe under HIP runtime settings (tools/micro/event_overhead.py, K=20).
set -o pipefail
mkdir -p gpurun_out/env
for v in "" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1" "HIP_FORCE_DEV_KERNARG=1" "ROC_ACTIVE_WAIT_TIMEOUT=0"; do
  echo "=== env: ${v:-default}" | tee -a gpurun_out/env/log.txt
  timeout -k 10 150 env $v python3 -u tools/micro/event_overhead.py 20 >> gpurun_out/env/log.txt 2>&1 || { echo "step failed $?" >> gpurun_out/env/log.txt; exit 1; }
done
