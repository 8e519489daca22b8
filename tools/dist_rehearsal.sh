#!/bin/bash
# Multi-rank rehearsal on ONE GPU (gloo exchange staged via host):
#  * config C: the candidate-sharded device episode over 2 and 4 ranks must log
#    exactly the same MPC steps as one rank over the same total candidates;
#  * config F: the leaf-sharded full tree over 2 ranks must return exactly the
#    same per-step results as one rank.
set -o pipefail
OUT=gpurun_out/${TAG:-dist}
mkdir -p $OUT
export MASTER_ADDR=127.0.0.1
# (no time-based ramp: every run logs the same first steps, which the
# 8192-record log ring still holds)
A="--cpu-seconds 0 --steps 40 --warmup 2 --dist-backend gloo --no-graph --no-second-pass --ramp-seconds 0"
F="--workload F --cpu-seconds 0 --steps 6 --warmup 1 --dist-backend gloo"
timeout -k 10 200 python bench.py $A --candidates-per-gpu 400000 --dump-log $OUT/w1.json > $OUT/w1.out 2>&1 && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py $A --gpus 2 --candidates-per-gpu 200000 --dump-log $OUT/w2.json > $OUT/w2.out 2>&1 && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 bench.py $A --gpus 4 --candidates-per-gpu 100000 --dump-log $OUT/w4.json > $OUT/w4.out 2>&1 && \
timeout -k 10 200 python bench.py $F --dump-log $OUT/f1.json > $OUT/f1.out 2>&1 && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py $F --gpus 2 --dump-log $OUT/f2.json > $OUT/f2.out 2>&1
rc=$?
python3 -c "
import json,sys
o='$OUT'
w1=json.load(open(o+'/w1.json')); w2=json.load(open(o+'/w2.json')); w4=json.load(open(o+'/w4.json'))
print('C steps', len(w1), len(w2), len(w4))
# one rank runs the chained kernel pass too (more real steps): compare the
# steps all three logged, aligned by step number
d1={r['step']: r for r in w1}
for name, w in (('w2', w2), ('w4', w4)):
    common=[r for r in w if r['step'] in d1]
    print('C', name, 'identical:', all(r == d1[r['step']] for r in common), ' over', len(common), 'steps')
f1=json.load(open(o+'/f1.json')); f2=json.load(open(o+'/f2.json'))
print('F steps', len(f1), len(f2), ' identical:', f1 == f2)
" || true
exit $rc
