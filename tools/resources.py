"""Per-kernel VGPRs / scratch / occupancy of the HIP library (hipcc remarks).
    python tools/resources.py [filter-regex]"""
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
       "-ffp-contract=off", "-I", os.path.join(REPO, "include"),
       "-Rpass-analysis=kernel-resource-usage", "-o", "/tmp/resources_probe.so",
       os.path.join(REPO, "diplomjourney_amd", "csrc", "mpc_rollout.hip")]
err = subprocess.run(cmd, capture_output=True, text=True, cwd="/tmp").stderr
pat = re.compile(sys.argv[1]) if len(sys.argv) > 1 else None
cur = None
for line in err.splitlines():
    m = re.search(r"remark: +(Function Name|VGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|"
                  r"LDS Size \[bytes/block\]|SGPRs Spill): (\S+)", line)
    if not m:
        continue
    k, v = m.groups()
    if k == "Function Name":
        cur = {"name": v}
    elif cur is not None:
        cur[k.split()[0]] = v
        if k.startswith("LDS"):
            if pat is None or pat.search(cur["name"]):
                print(f'{cur["name"][:90]:90s} vgpr {cur.get("VGPRs")} scratch {cur.get("ScratchSize")} '
                      f'occ {cur.get("Occupancy")} lds {cur.get("LDS")} sgpr-spill {cur.get("SGPRs")}')
            cur = None
