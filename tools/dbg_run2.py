"""Debug: the failing test's exact shape, repeated, with chain errors."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from diplomjourney_amd import math_model_tree as mmt  # noqa: E402
from diplomjourney_amd.episode import DeviceEpisode  # noqa: E402
from diplomjourney_amd.expansion import Expansion  # noqa: E402

eng = Expansion("cuda:0")
n, ns = int(sys.argv[1]), int(sys.argv[2])
K = int(sys.argv[3])
V = torch.tensor(mmt.vector_of_velocities(0.5), dtype=torch.float64, device="cuda")
B = torch.tensor(mmt.vector_of_beta_angles(0.0), dtype=torch.float64, device="cuda")
pool = [eng.sample_controls(V, B, n, ns, 500 + i) for i in range(8)]
b = [pool[i % 8] for i in range(K)]


def log(ep):
    return [(r.step, r.index, r.cost, r.x, r.p, r.episode) for r in ep.read_log()]


def mk():
    return DeviceEpisode(eng, n, ns, integrator="rect+cum", log_capacity=512, chain=True, L=0.5)


c = mk()
for x in b:
    c.step(controls=x)
c.flush()
want = log(c)
for rep in range(4):
    r = mk()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r.run(b)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    err = r.chain_error(local=True)
    got = log(r)
    bad = [i for i, (g, w) in enumerate(zip(got, want)) if g != w]
    print(f"rep {rep} K={K} {dt * 1e3:.2f} ms err {err} nbad {len(bad)} first {bad[:8]}", flush=True)
    if bad:
        i = bad[0]
        print("  got ", got[i:i + 2])
        print("  want", want[i:i + 2])
