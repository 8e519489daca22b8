# Same box: chained default vs two-launch rect+cum vs two-launch rect+rot (kernel and step times).
set -e
mkdir -p gpurun_out
for r in 1 2; do
  for a in "" "--no-chain" "--integrator rect+rot"; do
    echo "== $a" >> gpurun_out/cc.log
    timeout -k 10 240 python -u bench.py --cpu-seconds 0 --no-second-pass --steps 300 $a >> gpurun_out/cc.log 2>&1
  done
done
