#!/bin/bash
# A round's closing measurements on one GPU box (run from the repo root on the
# box).  Everything lands under gpurun_out/$TAG; every GPU step has its own
# time limit and the first failure ends the script.
#   PART=1: GPU suite, smoke, PMC traffic of the chained kernel (tiled
#           batches: config C, D per GPU, D in total) and of its P2P form,
#           the fp64 VALU counters of every kernel the line cites
#   PART=2: the default and driver-style bench lines, rocprof kernel stats of
#           the C-only run, the other workloads, the overlapped-exchange
#           teardown under memory-copy tracing
#   TAG=r06_close PART=1 bash tools/gpu_closing.sh
set -o pipefail
OUT=gpurun_out/${TAG:-closing}
mkdir -p $OUT
export TMPDIR=/tmp
step() {   # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "[closing] $name" >&2
  timeout -k 10 $secs "$@" || { echo "[closing] $name failed ($?)" >&2; exit 1; }
}
pmc() {    # pmc NAME "ARGS" ALGO_BYTES KERNEL_FILTER LABEL LAYOUT [tiled]
  local name=$1 args=$2 algo=$3 filt=$4 label=$5 layout=$6
  step pmc_$name 700 env MPC_LAYOUT=$layout TAG=${TAG:-closing}/pmc_$name ARGS="$args" \
    bash tools/pmc.sh > $OUT/pmc_$name.log 2>&1
  step pmc_${name}_sum 60 python3 tools/pmc_summary.py $OUT/pmc_$name $OUT/traffic_$name.json \
    $algo "$filt" "$label" $layout
}
if [ "${PART:-1}" = 1 ]; then
step tests 900 bash -c "TAG=${TAG:-closing}/tests bash tools/gpu_tests.sh"
step smoke 300 bash -c "python -c 'import __graft_entry__ as g; g.smoke()' > $OUT/smoke.txt 2>&1"
pmc chain_tiled "1000000 10 chain 20 4" 160e6 k_episode_chain k_episode_chain tiled
pmc chain_tiled_D "1250000 12 chain 20 4" 240e6 k_episode_chain k_episode_chain tiled
pmc chain_tiled_Dtotal "10000000 12 chain 12 4" 1920e6 k_episode_chain k_episode_chain tiled
pmc chain_p2p_tiled "1000000 10 p2p 20 4" 160e6 "k_episode_chain<1, 2, 4" "k_episode_chain[p2p]" tiled
step valu 900 bash -c "TAG=${TAG:-closing}/valu bash tools/pmc_valu.sh > $OUT/valu.log 2>&1"
fi
if [ "${PART:-2}" = 2 ]; then
step bench 300 bash -c "python bench.py > $OUT/bench.json 2> $OUT/bench.err"
step bench_driver 300 bash -c "python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err"
step rocprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/rocprof -o run -- python3 bench.py --cpu-seconds 0 --no-second-pass --no-config-d --parity-steps 0
find $OUT/rocprof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats_C.csv \;
for w in B D A R F G E; do
  step bench_$w 300 bash -c "python bench.py --cpu-seconds 0 --no-second-pass --workload $w > $OUT/bench_$w.json 2> $OUT/bench_$w.err"
done
step bench_qk21 300 bash -c "python bench.py --cpu-seconds 0 --no-second-pass --parity-steps 0 --no-config-d --integrator qk21 > $OUT/bench_qk21.json 2> $OUT/bench_qk21.err"
step bench_exchange 300 bash -c "python bench.py --cpu-seconds 0 --no-second-pass --parity-steps 0 --no-config-d --exchange > $OUT/bench_exchange.json 2> $OUT/bench_exchange.err"
step bench_exchange_rccl 300 bash -c "python bench.py --cpu-seconds 0 --no-second-pass --parity-steps 0 --no-config-d --exchange --exchange-mode rccl > $OUT/bench_exchange_rccl.json 2> $OUT/bench_exchange_rccl.err"
step overlap_exit 300 bash -c "rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $OUT/overlap_exit -o run -- python3 bench.py --exchange --overlap-exchange --cpu-seconds 0 --no-second-pass --parity-steps 0 --no-config-d --steps 20 --warmup 5 > $OUT/overlap_exit.log 2>&1"
fi
echo "[closing] done" >&2
