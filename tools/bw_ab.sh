# Block-wise persistent run (tools/var_bw.so) vs the in-tree run and the chained default.
# Variants first: bash tools/build_variant.sh bw (the in-tree source); bash tools/build_variant.sh bwstats -DMPC_RUN_STATS
set -e
mkdir -p gpurun_out
DIPLOMJOURNEY_MPC_LIB=tools/var_bw.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "run_" > gpurun_out/bw_tests.log 2>&1
for v in bw default; do
  lib=""; [ "$v" != default ] && lib=tools/var_$v.so
  env ${lib:+DIPLOMJOURNEY_MPC_LIB=$lib} timeout -k 10 120 python -u tools/time_run.py 1000000 10 200 3 >> gpurun_out/bw_time.log 2>&1
  env ${lib:+DIPLOMJOURNEY_MPC_LIB=$lib} timeout -k 10 120 python -u tools/time_run.py 8000000 10 60 2 >> gpurun_out/bw_time.log 2>&1
done
timeout -k 10 240 python -u bench.py --cpu-seconds 0 --no-second-pass > gpurun_out/bw_bench.log 2>&1
DIPLOMJOURNEY_MPC_LIB=tools/var_bw.so timeout -k 10 240 python -u bench.py --cpu-seconds 0 --no-second-pass --run >> gpurun_out/bw_bench.log 2>&1
DIPLOMJOURNEY_MPC_LIB=tools/var_bwstats.so timeout -k 10 120 python -u tools/unit_timeline.py 1000000 10 100 > gpurun_out/bw_tl.log 2>&1
