#!/bin/bash
# fp64 VALU counters (one pass of 8 SQ counters per kernel) for the VALU
# roofline of the kernels that are not HBM-bound: qk21's streaming kernel,
# the generated-controls rollout, the full-tree leaves; and the chained
# default for comparison.  Output: gpurun_out/$TAG/<name>/pmc1 + summaries.
set -o pipefail
OUT=gpurun_out/${TAG:-valu}
export MPC_LAYOUT=tiled   # the chained step on the bench default's tiled batches
mkdir -p $OUT
export TMPDIR=/tmp
CNT="SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_WAVES"
for spec in "chain|1000000 10 chain 20 4|k_episode_chain|160e6" \
            "qk21|1000000 10 qk21 20 4|k_rollout_argmin_stream|160e6" \
            "gen|1000000 10 generated 20 1|k_rollout_generated|0" \
            "ft|0 0 fulltree 6 1|k_ft_leaves|0" \
            "episodes_R|1000 1000 tree_episodes 1 1|k_episodes_run|0" \
            "ftepisodes_G|1000 50 ft_episodes 1 1|k_ftl_|0|sum"; do
  IFS='|' read name args kern algo mode <<< "$spec"
  mkdir -p $OUT/$name
  timeout -k 10 120 rocprofv3 --pmc $CNT --output-format csv -d $OUT/$name/pmc1 -o p -- python3 tools/prof_kernel.py $args > $OUT/$name/pmc1.log 2>&1 || { echo "$name failed"; tail -5 $OUT/$name/pmc1.log; exit 1; }
  python3 tools/pmc_summary.py $OUT/$name $OUT/$name.json $algo $kern $kern soa $mode > /dev/null || exit 1
done
python3 - <<PY
import json
for n in ("chain", "qk21", "gen", "ft", "episodes_R", "ftepisodes_G"):
    d = json.load(open("$OUT/%s.json" % n))
    c = d["counters_median_per_launch"]
    print(n, d["kernel"], "fp64 ops/launch %.4g" % (d["fp64_ops_per_launch"] or 0),
          {k: c.get(k) for k in ("SQ_INSTS_VALU", "SQ_INSTS_VALU_FLOPS_FP64", "SQ_INSTS_VALU_FLOPS_FP64_TRANS", "SQ_WAVES")})
PY
