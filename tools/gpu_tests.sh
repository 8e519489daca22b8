#!/bin/bash
# The GPU test suite on the box, one process, per-test timeout; output under
# gpurun_out/$TAG.  Extra pytest arguments (e.g. -k expr) pass through.
set -o pipefail
OUT=gpurun_out/${TAG:-gpu_tests}
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" > $OUT/pytest.log 2>&1
rc=$?
tail -30 $OUT/pytest.log
exit $rc
