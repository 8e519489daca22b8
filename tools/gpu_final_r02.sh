#!/bin/bash
# Round-2 closing check on one MI355X: GPU tests, smoke, the driver's bench
# command, the default bench, and the default bench under rocprofv3 stats.
# Each GPU step has its own limit; the steps are chained with &&.
set -o pipefail
O=gpurun_out/r02final
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err && \
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --cpu-seconds 0 > $O/bench_under_rocprof.json 2> $O/prof.err
rc=$?
tail -2 $O/pytest_gpu.log; tail -1 $O/smoke.log; cat $O/bench_driver.json | cut -c1-400
exit $rc
