#!/bin/bash
# Round 5 closing run on one GPU box, in two parts (each within one gpurun call).
#   PART=1: PMC traffic of the chained kernel over tiled batches (one-GPU and
#           P2P forms, configs C and D) and the fp64 VALU counters (pmc_valu.sh)
#   PART=2: the GPU suite (parity records), smoke(), the bench's default and
#           driver-style lines, rocprof kernel stats of the default workload
#           alone (no config-D sub-run, no parity leg: the same kernel instance),
#           and every other workload's line
#   TAG=name PART=1|2 bash tools/r05_close.sh
set -o pipefail
OUT=gpurun_out/${TAG:-r05c}
mkdir -p $OUT
export TMPDIR=/tmp
step() {   # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "[close] $name $(date +%T)"
  timeout -k 10 $secs "$@" || { echo "[close] $name failed ($?)"; exit 1; }
}
if [ "${PART:-1}" = 1 ]; then
for spec in "chain|1000000 10|chain|160e6|k_episode_chain<1, 2, 1|k_episode_chain|traffic_chain_tiled" \
            "chain_D|1250000 12|chain|240e6|k_episode_chain<1, 2, 1|k_episode_chain|traffic_chain_tiled_D" \
            "p2p|1000000 10|p2p|160e6|k_episode_chain<1, 2, 4|k_episode_chain[p2p]|traffic_chain_p2p_tiled" \
            "p2p_D|1250000 12|p2p|240e6|k_episode_chain<1, 2, 4|k_episode_chain[p2p]|traffic_chain_p2p_tiled_D"; do
  IFS='|' read name size mode algo filt label file <<< "$spec"
  step pmc_$name 300 bash -c "MPC_LAYOUT=tiled TAG=${TAG:-r05c}/pmc_$name ARGS='$size $mode 20 4' bash tools/pmc.sh > $OUT/pmc_$name.log 2>&1"
  step sum_$name 60 python3 tools/pmc_summary.py $OUT/pmc_$name $OUT/$file.json $algo "$filt" "$label" tiled
done
step valu 600 bash -c "MPC_LAYOUT=tiled TAG=${TAG:-r05c}/valu bash tools/pmc_valu.sh > $OUT/valu.log 2>&1"
tail -8 $OUT/valu.log
echo "[close] part 1 done $(date +%T)"
exit 0
fi
rm -f $OUT/parity.jsonl
step tests 900 env MPC_PARITY_REPORT=$OUT/parity.jsonl \
  python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
tail -2 $OUT/pytest.log
step smoke 120 bash -c "python -c 'import __graft_entry__ as g; g.smoke()' > $OUT/smoke.log 2>&1"
step bench 300 bash -c "python bench.py > $OUT/bench.json 2> $OUT/bench.err"
step bench_driver 300 bash -c "python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err"
step rocprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/rocprof -o run -- python3 bench.py --cpu-seconds 0 --no-second-pass --no-config-d --parity-steps 0
find $OUT/rocprof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
rm -rf $OUT/rocprof
for w in B D A E F G R; do
  step bench_$w 300 bash -c "python bench.py --cpu-seconds 0 --no-second-pass --workload $w > $OUT/bench_$w.json 2> $OUT/bench_$w.err"
done
step bench_qk21 300 bash -c "python bench.py --cpu-seconds 0 --no-second-pass --integrator qk21 --no-config-d > $OUT/bench_qk21.json 2> $OUT/bench_qk21.err"
step bench_exchange 300 bash -c "python bench.py --cpu-seconds 0 --no-second-pass --exchange --no-config-d > $OUT/bench_exchange.json 2> $OUT/bench_exchange.err"
step bench_exchange_rccl 300 bash -c "python bench.py --cpu-seconds 0 --no-second-pass --exchange --exchange-mode rccl --no-config-d > $OUT/bench_exchange_rccl.json 2> $OUT/bench_exchange_rccl.err"
python3 - <<PY
import json, glob
for f in sorted(glob.glob("$OUT/bench*.json")):
    try:
        d = json.loads([l for l in open(f) if l.startswith("{")][0])
    except Exception as e:
        print(f, "no line", e); continue
    r = d.get("roofline") or {}
    print(f.split("/")[-1], "%.4g %s" % (d["value"], d["unit"]), "ms/step %.5f" % d["ms_per_step"],
          "frac", r.get("frac"), "parity", (d.get("parity") or {}).get("identity_rate"))
PY
echo "[close] part 2 done $(date +%T)"
