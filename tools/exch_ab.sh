# One-rank rehearsal of the multi-GPU step structure (RCCL group of 1), both integrators.
set -e
mkdir -p gpurun_out
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29511
for a in "" "--integrator rect+cum"; do
  for r in 1 2; do
    echo "== exchange $a" >> gpurun_out/exch.log
    timeout -k 10 240 python -u bench.py --cpu-seconds 0 --no-second-pass --exchange $a >> gpurun_out/exch.log 2>&1
  done
done
