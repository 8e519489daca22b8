#!/bin/bash
# Round 5: the full-tree device episodes (workload G) — their tests, the G and
# R bench lines, and the VALU counters of both one-launch runs.
#   TAG=name bash tools/r05_g.sh
set -o pipefail
OUT=gpurun_out/${TAG:-r05g}
mkdir -p $OUT
export TMPDIR=/tmp
step() {   # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "[r05g] $name $(date +%T)"
  timeout -k 10 $secs "$@" || { echo "[r05g] $name failed ($?)"; exit 1; }
}
step tests 600 python -u -m pytest tests/test_fulltree_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
tail -3 $OUT/pytest.log
for w in G R; do
  step bench_$w 300 bash -c "python bench.py --cpu-seconds 0 --workload $w > $OUT/bench_$w.json 2> $OUT/bench_$w.err"
done
CNT="SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_WAVES"
for spec in "episodes_R|1000 1000 tree_episodes 1 1|k_episodes_run" \
            "ftepisodes_G|1000 50 ft_episodes 1 1|k_ft_episodes_run"; do
  IFS='|' read name args kern <<< "$spec"
  mkdir -p $OUT/valu/$name
  step pmc_$name 120 rocprofv3 --pmc $CNT --output-format csv -d $OUT/valu/$name/pmc1 -o p -- python3 tools/prof_kernel.py $args
  python3 tools/pmc_summary.py $OUT/valu/$name $OUT/valu/$name.json 0 $kern
done
echo "[r05g] done $(date +%T)"
