set -o pipefail
O=gpurun_out/b_modes; mkdir -p $O
for m in "chain:" "nochain:--no-chain" "fused:--no-chain --fused" "chain2:"; do
  n=${m%%:*}; a=${m#*:}
  timeout -k 10 200 python bench.py --workload B --cpu-seconds 0 --no-second-pass $a > $O/$n.out 2> $O/$n.err || { echo "$n failed"; tail -3 $O/$n.err; exit 1; }
  grep '^{' $O/$n.out | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('$n', round(d['ms_per_step']*1e3,2), 'kern', round(d['kernel_ms']*1e3,2), 'p50', d['p50_ms'], d['config']['step_launches'])"
done
