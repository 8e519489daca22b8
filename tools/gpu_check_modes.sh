#!/bin/bash
# One gpurun call: bench + rocprof stats of the chained (rect+cum) steps and
# of the persistent run.  Each GPU step has its own time limit; && chains them.
set -o pipefail
OUT=gpurun_out/${TAG:-modes}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --cpu-seconds 0 --integrator rect+cum > $OUT/bench_chain.json 2> $OUT/bench_chain.err && \
timeout -k 10 300 python bench.py --cpu-seconds 0 --integrator rect+cum --run > $OUT/bench_run.json 2> $OUT/bench_run.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_chain -o run -- python3 bench.py --cpu-seconds 0 --no-second-pass --integrator rect+cum > $OUT/bench_chain_prof.json 2> $OUT/prof_chain.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_run -o run -- python3 bench.py --cpu-seconds 0 --no-second-pass --integrator rect+cum --run > $OUT/bench_run_prof.json 2> $OUT/prof_run.err
rc=$?
echo "rc=$rc"
exit $rc
