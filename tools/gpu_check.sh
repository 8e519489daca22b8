#!/bin/bash
# One gpurun call: GPU tests, smoke, bench, rocprof stats.  Each GPU step has
# its own time limit; steps are chained with && so a failure stops the call.
set -o pipefail
OUT=gpurun_out/${TAG:-run}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -x -q -m gpu > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --cpu-seconds 0 ${BENCH_ARGS:-} > $OUT/bench_prof.json 2> $OUT/prof.err && \
if [ -n "${PMC:-}" ]; then TAG=${TAG:-run}/pmc ARGS="1000000 10 rect+rot 20 4" bash tools/pmc.sh > $OUT/pmc.log 2>&1 && \
  python3 tools/pmc_summary.py $OUT/pmc $OUT/traffic.json 160e6; fi
rc=$?
echo "rc=$rc"
tail -3 $OUT/pytest_gpu.log; cat $OUT/smoke.log; cat $OUT/bench.json
exit $rc
