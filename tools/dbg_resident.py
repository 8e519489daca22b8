import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np
import torch
from diplomjourney_amd import math_model_tree as mmt
from diplomjourney_amd.episode import DeviceEpisode
from diplomjourney_amd.expansion import Expansion
from diplomjourney_amd.abi import make_problem
eng = Expansion("cuda:0")
ep = DeviceEpisode(eng, 100_000, 10, integrator="rect+rot")
V = torch.tensor(mmt.vector_of_velocities(0.5), dtype=torch.float64, device="cuda")
B = torch.tensor(mmt.vector_of_beta_angles(0.0), dtype=torch.float64, device="cuda")
v, b = eng.sample_controls(V, B, ep.n_local, 10, 123, index_base=ep.lo)
torch.cuda.synchronize()
print("ptrs", hex(v.data_ptr()), hex(b.data_ptr()), hex(ep.v_sc.data_ptr()), v.stride(), ep.v_sc.stride())
ep.cur = (v, b)
ep.partials()
torch.cuda.synchronize()
recs = np.frombuffer(ep.ws.cpu().numpy().tobytes(), dtype=np.uint64).reshape(-1, 2)
print("resident recs", recs[:4].tolist())
ep.v_sc.copy_(v); ep.b_sc.copy_(b)
ep.cur = (ep.v_sc, ep.b_sc)
ep.partials()
torch.cuda.synchronize()
recs = np.frombuffer(ep.ws.cpu().numpy().tobytes(), dtype=np.uint64).reshape(-1, 2)
print("copied recs", recs[:4].tolist())
prob = make_problem(0.0, 0.0, 0.0, 2, 3, 0, 0, 0.5, 0.05, 0.1)
r = eng.fetch(eng.rollout_argmin(prob, v, b, integrator="rect+rot"))
print("plain api on pool tensors", r.cost, r.index)
