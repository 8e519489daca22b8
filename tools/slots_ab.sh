# Wave-wise run (MPC_RUN_BLOCKWISE=0) variants, built first with tools/build_variant.sh (e.g. pc3 -DMPC_RUN_BLOCKWISE=0 -DMPC_RUN_PER_CU=3)
set -e
mkdir -p gpurun_out
DIPLOMJOURNEY_MPC_LIB=tools/var_stats.so timeout -k 10 120 python -u tools/probe_run.py 1000000 10 100 > gpurun_out/probe_stats.log 2>&1
for v in pc3 s3r2pc3 s4pc2; do
  DIPLOMJOURNEY_MPC_LIB=tools/var_$v.so timeout -k 10 120 python -u tools/time_run.py 1000000 10 200 3 >> gpurun_out/slots_time2.log 2>&1
  DIPLOMJOURNEY_MPC_LIB=tools/var_$v.so timeout -k 10 120 python -u tools/time_run.py 8000000 10 60 2 >> gpurun_out/slots_time2.log 2>&1
done
