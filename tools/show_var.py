"""Condense tools/probe_gpu.py --time-only output (one line per timing)."""
import json
import sys

for line in sys.stdin:
    line = line.strip()
    if line.startswith("{"):
        d = json.loads(line)
        if d.get("check") == "time":
            print(f"   N={d['n_steps']:2d} C={d['n_cand']:8d} {d['integ']:9s} "
                  f"{d['ms'] * 1000:7.1f}us frac={d['frac_8TBs']}")
    elif line and not line.startswith("[gpurun] send"):
        print(line)
