#!/bin/bash
# Full tree after the criterion folding: GPU tests, F/G bench lines, fp64 VALU
# counters of k_ft_leaves (F) and k_ft_episodes_run (G).   TAG=name bash tools/r05_ft.sh
set -o pipefail
O=gpurun_out/${TAG:-ft5}; mkdir -p $O
export TMPDIR=/tmp
TAG=${TAG:-ft5} bash tools/ft_bench.sh || exit 1
CNT="SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_WAVES"
for spec in "ft|0 0 fulltree 6 1|k_ft_leaves|0" "ftepisodes_G|1000 50 ft_episodes 1 1|k_ft_episodes_run|0"; do
  IFS='|' read name args kern algo <<< "$spec"
  mkdir -p $O/$name
  timeout -k 10 120 rocprofv3 --pmc $CNT --output-format csv -d $O/$name/pmc1 -o p -- python3 tools/prof_kernel.py $args > $O/$name/pmc1.log 2>&1 || { echo "$name failed"; tail -5 $O/$name/pmc1.log; exit 1; }
  python3 tools/pmc_summary.py $O/$name $O/$name.json $algo $kern > /dev/null || exit 1
  python3 -c "import json; d=json.load(open('$O/$name.json')); c=d['counters_median_per_launch']; print('$name', 'VALU %.4g' % c['SQ_INSTS_VALU'], 'fp64 ops %.4g' % (d['fp64_ops_per_launch'] or 0))"
done
