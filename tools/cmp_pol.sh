# Interleaved A/B of library variants on config C (tools/var_<name>.so).
set -o pipefail
mkdir -p gpurun_out/pol
VARS=${VARS:-"p0 pnt psc1 pntsc"}
for rep in 1 2 3; do
for n in $VARS; do  # names: tools/var_<name>.so
  DIPLOMJOURNEY_MPC_LIB=tools/var_$n.so timeout -k 10 150 python bench.py --cpu-seconds 0 --steps 400 --warmup 20 > gpurun_out/pol/$n.$rep.json 2> gpurun_out/pol/$n.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/pol/$n.$rep.json').read().strip().splitlines()[-1]);print('$n', round(d['ms_per_step']*1e3,2), round(d['kernel_ms']*1e3,2), round(d['kernel_in_step_ms']*1e3,2))"
done; done
