#!/bin/bash
# Round 5 profiles on one GPU box: PMC traffic of the chained kernel at config
# D's per-GPU size (one-GPU form and P2P form), rocprof kernel stats of the
# default bench, and the overlapped exchange under a kernel + copy trace (the
# round-4 exit SIGSEGV) — it must exit 0.
#   TAG=name bash tools/r05_prof.sh
set -o pipefail
OUT=gpurun_out/${TAG:-r05p}
mkdir -p $OUT
export TMPDIR=/tmp
step() {   # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "[r05p] $name $(date +%T)"
  timeout -k 10 $secs "$@" || { echo "[r05p] $name failed ($?)"; exit 1; }
}
if [ -z "$SKIP_PMC" ]; then
step pmc_D 700 bash -c "TAG=${TAG:-r05p}/pmc_chain_D ARGS='1250000 12 chain 20 4' bash tools/pmc.sh > $OUT/pmc_chain_D.log 2>&1"
step pmc_D_sum 60 python3 tools/pmc_summary.py $OUT/pmc_chain_D $OUT/traffic_chain_D.json 240e6 "k_episode_chain<1, 2, 1" k_episode_chain
step pmc_p2p_D 700 bash -c "TAG=${TAG:-r05p}/pmc_p2p_D ARGS='1250000 12 p2p 20 4' bash tools/pmc.sh > $OUT/pmc_p2p_D.log 2>&1"
step pmc_p2p_D_sum 60 python3 tools/pmc_summary.py $OUT/pmc_p2p_D $OUT/traffic_chain_p2p_D.json 240e6 "k_episode_chain<1, 2, 4" "k_episode_chain[p2p]"
fi
step rocprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/rocprof -o run -- python3 bench.py --cpu-seconds 0 --no-second-pass
find $OUT/rocprof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
step overlap_trace 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/trace_ovl -o ovl -- python3 bench.py --exchange --overlap-exchange --cpu-seconds 0 --no-second-pass --steps 40 --warmup 5
echo "[r05p] overlap_trace exited 0"
rm -rf $OUT/trace_ovl $OUT/rocprof
echo "[r05p] done $(date +%T)"
