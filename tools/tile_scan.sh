# Rollout-kernel time vs candidate count around config C (tile-round effects).
set -e
mkdir -p gpurun_out
for n in 655360 983040 1000000 1310720 1638400 1966080 2621440; do
  timeout -k 10 120 python -u tools/ab_kernel.py $n 10 rect+cum >> gpurun_out/tile_scan.log 2>&1
done
