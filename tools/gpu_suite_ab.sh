#!/bin/bash
# Full GPU suite, then the exchange A/B (tools/p2p_ab.sh without its tests).
set -o pipefail
O=gpurun_out/${TAG:-suite}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
  > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
SKIP_TESTS=1 TAG=$TAG bash tools/p2p_ab.sh ${1:-1}
