#!/bin/bash
# Config C's chained step at several candidate counts per GPU (N = 10):
# how the fixed per-launch cost amortises.  K is scaled so the resident pool
# of distinct batches stays <= ~16 GB.  One JSON line per size.
set -o pipefail
O=gpurun_out/sweep
mkdir -p $O
: > $O/sweep.jsonl
for spec in 250000:500 500000:500 1000000:500 2000000:400 4000000:200 8000000:100; do
  n=${spec%%:*}; k=${spec##*:}
  timeout -k 10 240 python bench.py --cpu-seconds 0 --no-second-pass --candidates-per-gpu $n \
    --steps $k --warmup 20 >> $O/sweep.jsonl 2> $O/sweep_$n.err || exit 1
done
python - <<'PY'
import json
for l in open("gpurun_out/sweep/sweep.jsonl"):
    d = json.loads(l)
    c = d["config"]["candidates_per_gpu"]
    print(f'{c:>8} {d["value"]:.3e} rollouts/s  {d["ms_per_step"]*1e3:7.2f} us/step  '
          f'kernel {d["kernel_ms"]*1e3:7.2f} us  frac {d["roofline"]["frac"]:.3f}')
PY
