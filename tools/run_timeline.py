"""Per-step phases of the persistent run (a -DMPC_RUN_STATS build):
    python tools/with_lib.py tools/var_stats.so tools/run_timeline.py N NS K"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from diplomjourney_amd import math_model_tree as mmt, native  # noqa: E402
from diplomjourney_amd.episode import DeviceEpisode  # noqa: E402
from diplomjourney_amd.expansion import Expansion  # noqa: E402

n, ns, K = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
tiled = len(sys.argv) > 4 and sys.argv[4] == "tiled"
eng = Expansion("cuda:0")
V = torch.tensor(mmt.vector_of_velocities(0.5), dtype=torch.float64, device="cuda")
B = torch.tensor(mmt.vector_of_beta_angles(0.0), dtype=torch.float64, device="cuda")
smp = eng.sample_controls_tiled if tiled else eng.sample_controls
pool = [smp(V, B, n, ns, 500 + i) for i in range(min(K, 20))]
L = native.lib()
L.mpc_debug_run_stats.argtypes = [ctypes.c_void_p, ctypes.c_int]
ep = DeviceEpisode(eng, n, ns, integrator="rect+cum", log_capacity=4096, chain=True)
buf = np.zeros((64, 8), dtype=np.uint64)
for rep in range(3):
    L.mpc_debug_run_stats(None, 1)
    torch.cuda.synchronize()
    ep.run([pool[i % len(pool)] for i in range(K)])
    torch.cuda.synchronize()
    L.mpc_debug_run_stats(buf.ctypes.data, 0)
print("err", ep.chain_error())
t = buf.astype(np.int64)
base = t[0, 3]
us = lambda x: (x - base) / 100.0  # noqa: E731
print(" j  sel0   recs   done | u0    loopend waitend lastrec | poll_lat chain waited")
for j in range(K):
    r = t[j]
    print(f"{j:2d} {us(r[0]):6.1f} {us(r[1]):6.1f} {us(r[2]):6.1f} | {us(r[3]):6.1f} {us(r[4]):6.1f}"
          f" {us(r[5]):6.1f} {us(r[6]):6.1f} | {(r[1]-r[6])/100:5.2f} {(r[2]-r[1])/100:5.2f} {r[7]}")
