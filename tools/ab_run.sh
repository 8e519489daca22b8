# A/B of the persistent run variants against the per-step launch paths (one GPU box call).
#   bash tools/ab_run.sh "variant ..."   (tools/var_<variant>.so; "default" = the in-tree library)
# Variants first: bash tools/build_variant.sh NAME -D... (e.g. stats -DMPC_RUN_STATS; the wave-wise design is in the history: commit 50b37c6)
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "run_" > gpurun_out/ab_tests.log 2>&1
for v in $1; do
  lib=""; [ "$v" != default ] && lib=tools/var_$v.so
  env ${lib:+DIPLOMJOURNEY_MPC_LIB=$lib} timeout -k 10 120 python -u tools/time_run.py 1000000 10 200 3 >> gpurun_out/ab_time.log 2>&1
  env ${lib:+DIPLOMJOURNEY_MPC_LIB=$lib} timeout -k 10 120 python -u tools/time_run.py 8000000 10 60 2 >> gpurun_out/ab_time.log 2>&1
done
for a in "--integrator rect+cum" "--integrator rect+cum --run"; do
  echo "== bench $a" >> gpurun_out/ab_bench.log
  timeout -k 10 240 python -u bench.py --cpu-seconds 0 --no-second-pass $a >> gpurun_out/ab_bench.log 2>&1
done
DIPLOMJOURNEY_MPC_LIB=tools/var_stats.so timeout -k 10 120 python -u tools/unit_timeline.py 1000000 10 100 > gpurun_out/ab_tl.log 2>&1
