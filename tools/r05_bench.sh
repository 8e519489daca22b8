#!/bin/bash
# Round 5: bench-focused check — the bench tests, the default and driver-style
# lines, and the rocprof kernel stats of the default bench.
#   TAG=name bash tools/r05_bench.sh
set -o pipefail
OUT=gpurun_out/${TAG:-r05b}
mkdir -p $OUT
export TMPDIR=/tmp
step() {   # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "[r05b] $name $(date +%T)"
  timeout -k 10 $secs "$@" || { echo "[r05b] $name failed ($?)"; exit 1; }
}
step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "${TESTS:-bench or two_ranks}" > $OUT/pytest.log 2>&1
tail -2 $OUT/pytest.log
step bench 300 bash -c "python bench.py > $OUT/bench.json 2> $OUT/bench.err"
step bench_driver 300 bash -c "python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err"
step rocprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/rocprof -o run -- python3 bench.py --cpu-seconds 0 --no-second-pass
find $OUT/rocprof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
rm -rf $OUT/rocprof
python3 - <<PY
import json
def line(f):
    return json.loads([l for l in open(f) if l.startswith("{")][0])
for f in ("bench", "bench_driver"):
    d = line("$OUT/%s.json" % f)
    cd = d.get("config_d") or {}
    print(f, "C %.2f us/step kernel %.2f us (sustained %s) frac %.3f ceiling %.2f us" % (
        d["ms_per_step"] * 1e3, d["kernel_ms"] * 1e3, d.get("kernel_ms_sustained"),
        d["roofline"]["frac"], d["roofline"]["stream_ceiling_ms"] * 1e3),
        "| D %.2f us/step kernel %.2f frac %.3f" % (cd.get("ms_per_step", 0) * 1e3,
        cd.get("kernel_ms", 0) * 1e3, (cd.get("roofline") or {}).get("frac", 0)),
        "| parity", d.get("parity", {}).get("identity_rate"), "p50_host", d.get("p50_host_ms"))
PY
head -3 $OUT/kernel_stats.csv | cut -c1-160
echo "[r05b] done $(date +%T)"
