set -o pipefail
O=gpurun_out/r06/rab; mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for v in ep0 ep1; do
    timeout -k 10 200 python tools/with_lib.py tools/var_$v.so bench.py --workload R --cpu-seconds 0 > $O/$v.$rep.json 2> $O/$v.$rep.err || { echo $v failed; tail -5 $O/$v.$rep.err; exit 1; }
  done
  timeout -k 10 200 python bench.py --workload R --cpu-seconds 0 > $O/ep2.$rep.json 2> $O/ep2.$rep.err || { echo ep2 failed; tail -5 $O/ep2.$rep.err; exit 1; }
done
timeout -k 10 600 python -u -m pytest tests/test_fulltree_gpu.py -x -q --timeout 300 --timeout-method thread -k "tree_episode or robot_0 or chunked" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/ovl -o run -- python3 bench.py --exchange --overlap-exchange --cpu-seconds 0 --no-second-pass --parity-steps 0 --no-config-d --steps 20 --warmup 5 > $O/ovl.log 2>&1
echo ovl rc=$?
