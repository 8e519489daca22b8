#!/bin/bash
# Counter passes for the rollout kernel (one counter group per pass; PMC runs
# never combine with sys/runtime traces).  Output under gpurun_out/$TAG/pmc*.
#   TAG=name ARGS="n_cand n_steps integ reps" bash tools/pmc.sh
OUT=gpurun_out/${TAG:-pmc}
mkdir -p $OUT
export TMPDIR=/tmp
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES" \
           "SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
           "FETCH_SIZE" "WRITE_SIZE" \
           "GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY SQ_INSTS_LDS" \
           ${EXTRA_GROUPS:-}; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc$i -o p -- python3 tools/prof_kernel.py ${ARGS:-} > $OUT/pmc$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/pmc$i.log; }
done
ls -R $OUT | head -50
# summary: KERNEL=k_episode_chain ARGS="1000000 10 chain 20 4" for the chained step
