#!/bin/bash
# A round's closing measurements on one GPU box (run from the repo root on the
# box): GPU suite, smoke, the bench's default and driver-style lines, rocprof
# kernel stats of the default bench, PMC traffic + VALU passes of the chained
# kernel, and the other workloads.  Everything lands under gpurun_out/$TAG;
# every GPU step has its own time limit and the first failure ends the script.
#   TAG=r04_close bash tools/gpu_closing.sh
set -o pipefail
OUT=gpurun_out/${TAG:-closing}
mkdir -p $OUT
export TMPDIR=/tmp
step() {   # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "[closing] $name" >&2
  timeout -k 10 $secs "$@" || { echo "[closing] $name failed ($?)" >&2; exit 1; }
}
# PART=1: tests, smoke, default bench + rocprof + PMC; PART=2: the rest (one
# gpurun call each stays within its time limit); unset: both.
if [ "${PART:-1}" = 1 ] || [ -z "$PART" ]; then
step tests 900 bash -c "TAG=${TAG:-closing}/tests bash tools/gpu_tests.sh"
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 300 bash -c "python bench.py > $OUT/bench.json 2> $OUT/bench.err"
step bench_driver 200 bash -c "python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err"
step rocprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/rocprof -o run -- python3 bench.py --cpu-seconds 0 --no-second-pass
cp $OUT/rocprof/*/run_kernel_stats.csv $OUT/kernel_stats.csv 2>/dev/null || find $OUT/rocprof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
step pmc 700 bash -c "TAG=${TAG:-closing}/pmc_chain ARGS='1000000 10 chain 20 4' bash tools/pmc.sh > $OUT/pmc_chain.log 2>&1"
step pmc_sum 60 python3 tools/pmc_summary.py $OUT/pmc_chain $OUT/traffic_chain.json 160e6 k_episode_chain
step valu 600 bash -c "TAG=${TAG:-closing}/valu bash tools/pmc_valu.sh > $OUT/valu.log 2>&1"
fi
if [ "${PART:-2}" = 2 ] || [ -z "$PART" ]; then
step pmc_p2p 700 bash -c "TAG=${TAG:-closing}/pmc_p2p ARGS='1000000 10 p2p 20 4' bash tools/pmc.sh > $OUT/pmc_p2p.log 2>&1"
step pmc_p2p_sum 60 python3 tools/pmc_summary.py $OUT/pmc_p2p $OUT/traffic_chain_p2p.json 160e6 "k_episode_chain<1, 2, 4" "k_episode_chain[p2p]"
for w in B D A R F G E; do
  step bench_$w 300 bash -c "python bench.py --cpu-seconds 0 --no-second-pass --workload $w > $OUT/bench_$w.json 2> $OUT/bench_$w.err"
done
step bench_qk21 300 bash -c "python bench.py --cpu-seconds 0 --no-second-pass --integrator qk21 > $OUT/bench_qk21.json 2> $OUT/bench_qk21.err"
step bench_exchange 300 bash -c "python bench.py --cpu-seconds 0 --no-second-pass --exchange > $OUT/bench_exchange.json 2> $OUT/bench_exchange.err"
step bench_exchange_rccl 300 bash -c "python bench.py --cpu-seconds 0 --no-second-pass --exchange --exchange-mode rccl > $OUT/bench_exchange_rccl.json 2> $OUT/bench_exchange_rccl.err"
step rocprof_p2p 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/rocprof_p2p -o run -- python3 bench.py --cpu-seconds 0 --no-second-pass --exchange
find $OUT/rocprof_p2p -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats_p2p.csv \;
fi
echo "[closing] done" >&2
