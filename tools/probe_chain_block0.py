"""Developer probe: stage times of the chained launch's block 0 (the previous
step's completion) while the launch's tiles stream, from a library built with
-DMPC_FIN_TRACE (10-ns s_memrealtime ticks in the result record's traj[30..31]).
    tools/build_variant.sh fin -DMPC_FIN_TRACE
    DIPLOMJOURNEY_MPC_LIB=tools/var_fin.so python tools/probe_chain_block0.py"""
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
ep = DeviceEpisode(eng, 1_000_000, 10, integrator="rect+cum", chain=True)
V = torch.tensor(mmt.vector_of_velocities(0.5), dtype=torch.float64, device="cuda")
B = torch.tensor(mmt.vector_of_beta_angles(0.0), dtype=torch.float64, device="cuda")
pool = [eng.sample_controls(V, B, ep.n_local, 10, 300 + i) for i in range(8)]
for i in range(300):
    ep.step(controls=pool[i % 8])
rows = []
for i in range(40):
    ep.step(controls=pool[i % 8])
    torch.cuda.synchronize()
    r = result_from_bytes(ep.local.cpu().numpy().tobytes())
    rows.append([r.traj[31][0], r.traj[31][1], r.traj[31][2], r.traj[30][0], r.traj[30][1],
                 r.traj[30][2]])
ep.flush()
a = np.array(rows) * 0.01
print("chained block 0 stages (us, median): records+reduce %.2f  winner re-roll %.2f  "
      "update %.2f (copy-in %.2f, advance %.2f, prepare %.2f)" % tuple(np.median(a, axis=0)))
