#!/bin/bash
# Round 5, tiled layout: PMC traffic of the chained kernel over tiled batches
# (one-GPU and P2P forms, configs C and D), the GPU suite, the bench's default
# and driver-style lines, and a same-box A/B of the layouts.
#   TAG=name bash tools/r05_tiled.sh
set -o pipefail
OUT=gpurun_out/${TAG:-r05t}
mkdir -p $OUT profiles/r05
export TMPDIR=/tmp
step() {   # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "[r05t] $name $(date +%T)"
  timeout -k 10 $secs "$@" || { echo "[r05t] $name failed ($?)"; exit 1; }
}
if [ -z "$SKIP_PMC" ]; then
for spec in "chain|1000000 10|chain|160e6|k_episode_chain<1, 2, 1|k_episode_chain|traffic_chain_tiled" \
            "chain_D|1250000 12|chain|240e6|k_episode_chain<1, 2, 1|k_episode_chain|traffic_chain_tiled_D" \
            "p2p|1000000 10|p2p|160e6|k_episode_chain<1, 2, 4|k_episode_chain[p2p]|traffic_chain_p2p_tiled" \
            "p2p_D|1250000 12|p2p|240e6|k_episode_chain<1, 2, 4|k_episode_chain[p2p]|traffic_chain_p2p_tiled_D"; do
  IFS='|' read name size mode algo filt label file <<< "$spec"
  step pmc_$name 700 bash -c "MPC_LAYOUT=tiled TAG=${TAG:-r05t}/pmc_$name ARGS='$size $mode 20 4' bash tools/pmc.sh > $OUT/pmc_$name.log 2>&1"
  step sum_$name 60 python3 tools/pmc_summary.py $OUT/pmc_$name $OUT/$file.json $algo "$filt" "$label" tiled
  cp $OUT/$file.json profiles/r05/
done
fi
rm -f $OUT/parity.jsonl
step tests 1000 env MPC_PARITY_REPORT=$OUT/parity.jsonl \
  python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
tail -2 $OUT/pytest.log
step bench 300 bash -c "python bench.py > $OUT/bench.json 2> $OUT/bench.err"
step bench_driver 300 bash -c "python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err"
for r in 1 2 3; do
  for lay in tiled soa; do
    step ab_$lay$r 300 bash -c "python bench.py --cpu-seconds 0 --no-second-pass --parity-steps 0 --no-config-d --layout $lay > $OUT/ab_$lay$r.json 2> $OUT/ab_$lay$r.err"
  done
done
python3 - <<PY
import json
def line(f):
    return json.loads([l for l in open(f) if l.startswith("{")][0])
for f in ("bench", "bench_driver"):
    d = line("$OUT/%s.json" % f)
    cd = d.get("config_d") or {}
    print(f, "C %.2f us/step kernel %.2f us frac %.3f traffic %s ceiling %.1f" % (
        d["ms_per_step"] * 1e3, d["kernel_ms"] * 1e3, d["roofline"]["frac"], d["roofline"]["traffic"],
        d["roofline"]["stream_ceiling_GBs"]),
        "| D %.2f us/step frac %.3f" % (cd.get("ms_per_step", 0) * 1e3, (cd.get("roofline") or {}).get("frac", 0)),
        "| parity", d.get("parity", {}).get("identity_rate"))
for r in (1, 2, 3):
    for lay in ("tiled", "soa"):
        d = line("$OUT/ab_%s%d.json" % (lay, r))
        print("ab", lay, r, "step %.2f kernel %.2f us frac %.3f ceiling %.2f us" % (
            d["ms_per_step"] * 1e3, d["kernel_ms"] * 1e3, d["roofline"]["frac"],
            d["roofline"]["stream_ceiling_ms"] * 1e3))
PY
echo "[r05t] done $(date +%T)"
