import os, sys, time
sys.path.insert(0, '/root/repo')
import torch
from diplomjourney_amd import math_model_tree as mmt
from diplomjourney_amd.episode import DeviceEpisode
from diplomjourney_amd.expansion import Expansion
eng = Expansion("cuda:0")
V = torch.tensor(mmt.vector_of_velocities(0.5), dtype=torch.float64, device="cuda")
B = torch.tensor(mmt.vector_of_beta_angles(0.0), dtype=torch.float64, device="cuda")
pool = [eng.sample_controls(V, B, 1000000, 10, 0x5EED + i) for i in range(8)]
ep = DeviceEpisode(eng, 1000000, 10, integrator="rect+cum", chain=True, log_capacity=8192)
for i in range(50): ep.step(controls=pool[i % 8])
torch.cuda.synchronize()
for trial in range(3):
    t0 = time.perf_counter()
    for i in range(200): ep.step(controls=pool[i % 8])
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"host enqueue {((t1-t0)/200)*1e6:.1f} us/step, wall {((t2-t0)/200)*1e6:.1f} us/step")
ev = torch.cuda.Event()
t0 = time.perf_counter()
for i in range(1000): ev.record()
print(f"event record {(time.perf_counter()-t0)/1000*1e6:.1f} us")
