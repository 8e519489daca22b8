#!/bin/bash
# Same-box A/B of the in-tree library against tools/var_$1.so at configs C and
# B (tools/ab_chain.py, ROUNDS interleaved rounds), after the GPU test suite.
#   TAG=name bash tools/ab_run.sh VARIANT [ROUNDS]
set -o pipefail
O=gpurun_out/${TAG:-ab}; mkdir -p $O
R=${2:-3}
timeout -k 10 400 python tools/ab_chain.py $R - tools/var_$1.so > $O/ab_C.txt 2>&1 &&
AB_N=100000 AB_NS=3 timeout -k 10 300 python tools/ab_chain.py $R - tools/var_$1.so > $O/ab_B.txt 2>&1
rc=$?
cat $O/ab_C.txt $O/ab_B.txt
exit $rc
