#!/bin/bash
# One GPU box pass during development: the GPU suite (or the -k subset in
# $K), then the default bench line and the exchange / B lines.  Output under
# gpurun_out/$TAG; every GPU step has its own limit, the first failure ends it.
#   TAG=r04b K="expr" bash tools/gpu_quick.sh
set -o pipefail
OUT=gpurun_out/${TAG:-quick}
mkdir -p $OUT
export TMPDIR=/tmp
step() {   # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "[quick] $name $(date +%T)" >&2
  timeout -k 10 $secs "$@" || { echo "[quick] $name failed ($?)" >&2; exit 1; }
}
if [ -n "${K:-}" ]; then
  step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" -p no:cacheprovider > $OUT/pytest.log 2>&1
elif [ -z "${NOTESTS:-}" ]; then
  step tests 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
fi
tail -3 $OUT/pytest.log 2>/dev/null
step bench 300 bash -c "python bench.py --cpu-seconds 0 > $OUT/bench.json 2> $OUT/bench.err"
step bench_xchg 300 bash -c "python bench.py --cpu-seconds 0 --no-second-pass --exchange > $OUT/bench_exchange.json 2> $OUT/bench_exchange.err"
step bench_B 300 bash -c "python bench.py --cpu-seconds 0 --no-second-pass --workload B > $OUT/bench_B.json 2> $OUT/bench_B.err"
python3 - <<PY
import json
for n in ("bench", "bench_exchange", "bench_B"):
    try:
        d = json.loads([l for l in open("$OUT/%s.json" % n) if l.startswith("{")][0])
    except Exception as e:
        print(n, "no line", e); continue
    r = d.get("roofline") or {}
    print(n, "value %.4g" % d["value"], "ms/step %.5f" % d["ms_per_step"], "kernel_ms", d.get("kernel_ms"),
          "frac", r.get("frac"), "chain_error", d.get("chain_error"))
PY
echo "[quick] done" >&2
