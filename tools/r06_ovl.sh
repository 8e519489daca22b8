set -o pipefail
O=gpurun_out/r06/ovl; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/ovl -o run -- python3 bench.py --exchange --overlap-exchange --cpu-seconds 0 --no-second-pass --parity-steps 0 --no-config-d --steps 20 --warmup 5 > $O/ovl.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/def -o run -- python3 bench.py --cpu-seconds 0 --no-second-pass --parity-steps 0 --no-config-d --steps 20 --warmup 5 > $O/def.log 2>&1 || exit 1
grep -c callback $O/ovl.log $O/def.log
timeout -k 10 200 python tools/episodes_timeline.py run 1000 1000 > $O/tl_R.txt 2>&1
