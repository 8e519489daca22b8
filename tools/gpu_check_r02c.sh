#!/bin/bash
# Round-2 default (chained rect+cum) check: GPU tests, smoke, benches of the
# episode workloads, rocprof stats of the default bench, PMC passes of the
# chained kernel.  Each GPU step has its own time limit; && chains them.
set -o pipefail
OUT=gpurun_out/${TAG:-r02c}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -x -q -m gpu > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err && \
timeout -k 10 300 python bench.py --cpu-seconds 0 --no-second-pass --workload B > $OUT/bench_B.json 2> $OUT/bench_B.err && \
timeout -k 10 300 python bench.py --cpu-seconds 0 --no-second-pass --workload D > $OUT/bench_D.json 2> $OUT/bench_D.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --cpu-seconds 0 > $OUT/bench_prof.json 2> $OUT/prof.err && \
TAG=${TAG:-r02c}/pmc ARGS="1000000 10 chain 20 4" bash tools/pmc.sh > $OUT/pmc.log 2>&1 && \
python3 tools/pmc_summary.py $OUT/pmc $OUT/traffic_chain.json 160e6 k_episode_chain
rc=$?
echo "rc=$rc"
tail -2 $OUT/pytest_gpu.log; cat $OUT/smoke.log
exit $rc
