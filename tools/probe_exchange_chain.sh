#!/bin/bash
# Multi-GPU step structure rehearsed on ONE GPU over a 1-rank nccl group,
# graph-captured: two-launch rect+rot (rollout, finalize, all_gather, advance)
# vs chained rect+cum (chain launch = rollout + advance of the previous step,
# then finalize, all_gather), each against its single-GPU step.
set -o pipefail
OUT=gpurun_out/${TAG:-xchain}
mkdir -p $OUT
export MASTER_ADDR=127.0.0.1 TMPDIR=/tmp
A="--cpu-seconds 0 --no-second-pass --steps ${K:-500}"
for integ in rect+rot rect+cum; do
  timeout -k 10 150 python bench.py $A --integrator $integ > $OUT/single_$integ.out 2> $OUT/single_$integ.err || exit 1
  timeout -k 10 150 python bench.py $A --integrator $integ --exchange > $OUT/xg_$integ.out 2> $OUT/xg_$integ.err || exit 1
done
python3 - "$OUT" <<'PY'
import json, sys
o = sys.argv[1]
for integ in ("rect+rot", "rect+cum"):
    for n in ("single", "xg"):
        d = json.loads(open(f"{o}/{n}_{integ}.out").read().strip().splitlines()[-1])
        print(integ, n, round(d["ms_per_step"] * 1e3, 2), "us/step", d["config"]["step_launches"])
PY
