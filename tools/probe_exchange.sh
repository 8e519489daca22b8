#!/bin/bash
# Exchange-path rehearsal on ONE GPU: the multi-GPU step structure (finalize ->
# RCCL all_gather over a 1-rank nccl group -> advance), eager and captured in a
# HIP graph, against the single-GPU step; the device episode logs must match.
set -o pipefail
OUT=gpurun_out/${TAG:-xchg}
mkdir -p $OUT
export MASTER_ADDR=127.0.0.1 TMPDIR=/tmp
A="--cpu-seconds 0 --no-second-pass --steps ${K:-300}"
timeout -k 10 150 python bench.py $A --dump-log $OUT/single.json > $OUT/single.out 2> $OUT/single.err && \
timeout -k 10 150 python bench.py $A --no-graph > $OUT/single_eager.out 2> $OUT/single_eager.err && \
timeout -k 10 150 python bench.py $A --exchange --dump-log $OUT/xg.json > $OUT/xg.out 2> $OUT/xg.err && \
timeout -k 10 150 python bench.py $A --exchange --no-graph --dump-log $OUT/xe.json > $OUT/xe.out 2> $OUT/xe.err
rc=$?
python3 - "$OUT" <<'PY' || true
import json, sys
o = sys.argv[1]
for n in ("single", "single_eager", "xg", "xe"):
    try:
        d = json.loads(open(f"{o}/{n}.out").read().strip().splitlines()[-1])
        print(n, "%.4g rollouts/s" % d["value"], "%.2f us/step" % (d["ms_per_step"] * 1e3),
              "p50 %.1f us" % (d["p50_ms"] * 1e3), d["config"]["launch"])
    except Exception as e:
        print(n, "no result", e)
try:
    s, xg, xe = (json.load(open(f"{o}/{n}.json")) for n in ("single", "xg", "xe"))
    # the eager run has no untimed first graph replay: compare its prefix
    print("logs", len(s), len(xg), len(xe), "xg==single", s == xg,
          "xe==single[:len(xe)]", s[:len(xe)] == xe)
except Exception as e:
    print("log compare failed", e)
PY
exit $rc
