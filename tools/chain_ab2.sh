# Chained-step A/B: in-tree library vs tools/var_c4pin.so, interleaved, after the chain tests.
# Variants first: bash tools/build_variant.sh c4pin -DMPC_CHAIN_WAVES=4 -DMPC_CHAIN_PIN=true; var_old.so = a build of an earlier commit
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "chain" > gpurun_out/cab_tests.log 2>&1
for r in 1 2; do
  for v in default old c4pin; do
    lib=""; [ "$v" != default ] && lib=tools/var_$v.so
    echo "== $v" >> gpurun_out/cab_bench.log
    env ${lib:+DIPLOMJOURNEY_MPC_LIB=$lib} timeout -k 10 240 python -u bench.py --cpu-seconds 0 --no-second-pass --integrator rect+cum >> gpurun_out/cab_bench.log 2>&1
  done
done
