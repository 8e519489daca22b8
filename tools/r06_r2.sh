set -o pipefail
O=gpurun_out/r06/r2; mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  timeout -k 10 200 python bench.py --workload R --cpu-seconds 0 > $O/new.$rep.json 2> $O/new.$rep.err || { echo new failed; tail -5 $O/new.$rep.err; exit 1; }
done
timeout -k 10 600 python -u -m pytest tests/test_fulltree_gpu.py -x -q --timeout 300 --timeout-method thread -k "tree_episode or robot_0 or chunked" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python tools/episodes_timeline.py run 1000 1000 > $O/tl_R.txt 2>&1
