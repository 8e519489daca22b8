#!/bin/bash
# Time every tools/var_*.so kernel variant, one process each (gpurun helper).
mkdir -p gpurun_out
for so in tools/var_*.so; do
  DIPLOMJOURNEY_MPC_LIB=$so timeout -k 10 120 python tools/probe_gpu.py --time-only 2>/dev/null | grep -v amdgpu.ids || exit 1
done
