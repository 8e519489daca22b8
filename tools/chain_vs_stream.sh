# Same box: the rect+cum stream kernel alone (ab_kernel) vs the chained launch (bench chain_pass).
set -e
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 120 python -u tools/ab_kernel.py 1000000 10 rect+cum >> gpurun_out/cvs.log 2>&1
  timeout -k 10 240 python -u bench.py --cpu-seconds 0 --no-second-pass --steps 200 >> gpurun_out/cvs.log 2>&1
done
