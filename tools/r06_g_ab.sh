set -o pipefail
O=gpurun_out/r06/gab; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_fulltree_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2; do
  timeout -k 10 200 python tools/with_lib.py tools/var_ft0.so bench.py --workload G --cpu-seconds 0 > $O/ft0.$rep.json 2> $O/ft0.$rep.err || { echo ft0 failed; tail -5 $O/ft0.$rep.err; exit 1; }
  timeout -k 10 200 python bench.py --workload G --cpu-seconds 0 > $O/new.$rep.json 2> $O/new.$rep.err || { echo new failed; tail -5 $O/new.$rep.err; exit 1; }
done
