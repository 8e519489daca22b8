"""Developer probe: stage times inside k_finalize (library built with
-DMPC_FIN_TRACE; 10-ns s_memrealtime ticks written to traj[31])."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from diplomjourney_amd import math_model_tree as mmt  # noqa: E402
from diplomjourney_amd.abi import result_from_bytes  # noqa: E402
from diplomjourney_amd.episode import DeviceEpisode  # noqa: E402
from diplomjourney_amd.expansion import Expansion  # noqa: E402

eng = Expansion("cuda:0")
ep = DeviceEpisode(eng, 1_000_000, 10, integrator="rect+rot")
V = torch.tensor(mmt.vector_of_velocities(0.5), dtype=torch.float64, device="cuda")
B = torch.tensor(mmt.vector_of_beta_angles(0.0), dtype=torch.float64, device="cuda")
pool = [eng.sample_controls(V, B, ep.n_local, 10, 300 + i) for i in range(4)]
rows = []
for i in range(30):
    ep.step(controls=pool[i % 4])
    torch.cuda.synchronize()
    r = result_from_bytes(ep.local.cpu().numpy().tobytes())
    rows.append([r.traj[31][0], r.traj[31][1], r.traj[31][2], r.traj[30][0], r.traj[30][1], r.traj[30][2]])
a = np.array(rows[5:]) * 0.01
print("finalize stages (us): reduce+H %.2f  emit %.2f  hook %.2f "
      "(copy-in %.2f, advance %.2f, prepare %.2f)" % tuple(np.median(a, axis=0)))
