#!/bin/bash
# Round 5 checkpoint on one GPU box: the GPU suite (parity records to
# $OUT/parity.jsonl), then the bench's default line and the driver-style line.
#   TAG=name bash tools/r05_check.sh [pytest args]
set -o pipefail
OUT=gpurun_out/${TAG:-r05}
mkdir -p $OUT
export TMPDIR=/tmp
step() {   # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "[r05] $name $(date +%T)"
  timeout -k 10 $secs "$@" || { echo "[r05] $name failed ($?)"; exit 1; }
}
rm -f $OUT/parity.jsonl
step tests 1000 env MPC_PARITY_REPORT=$OUT/parity.jsonl \
  python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" \
  > $OUT/pytest.log 2>&1
tail -3 $OUT/pytest.log
[ -n "$NO_BENCH" ] && exit 0
step bench 300 bash -c "python bench.py > $OUT/bench.json 2> $OUT/bench.err"
step bench_driver 300 bash -c "python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err"
python3 - <<EOF
import json
for f in ("bench", "bench_driver"):
    d = json.loads([l for l in open("$OUT/%s.json" % f) if l.startswith("{")][0])
    cd = d.get("config_d") or {}
    print(f, "C %.2f us/step frac %.3f" % (d["ms_per_step"] * 1e3, d["roofline"]["frac"]),
          "| D %.2f us/step frac %.3f" % (cd.get("ms_per_step", 0) * 1e3, (cd.get("roofline") or {}).get("frac", 0)),
          "| parity", d.get("parity", {}).get("identity_rate"), d.get("parity", {}).get("check_s"))
EOF
echo "[r05] done $(date +%T)"
