"""Debug probe for the persistent run (mpc_episode_run): chained vs run logs on
a few steps, with single-step runs and a repeated-batch run as controls."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from diplomjourney_amd import math_model_tree as mmt  # noqa: E402
from diplomjourney_amd.episode import DeviceEpisode  # noqa: E402
from diplomjourney_amd.expansion import Expansion  # noqa: E402

eng = Expansion("cuda:0")
n, ns = int(sys.argv[1]) if len(sys.argv) > 1 else 50_000, 10
V = torch.tensor(mmt.vector_of_velocities(0.5), dtype=torch.float64, device="cuda")
B = torch.tensor(mmt.vector_of_beta_angles(0.0), dtype=torch.float64, device="cuda")
pool = [eng.sample_controls(V, B, n, ns, 500 + i) for i in range(4)]


def log(ep):
    return [(r.step, r.index, round(r.cost, 6), round(r.x, 6), r.p, r.episode)
            for r in ep.read_log()]


def mk():
    return DeviceEpisode(eng, n, ns, integrator="rect+cum", log_capacity=64, chain=True)


batches = [pool[i % 4] for i in range(4)]
ch = mk()
for c in batches:
    ch.step(controls=c)
ch.flush()
print("chain ", log(ch))
r1 = mk()
for c in batches:
    r1.run([c])
print("run1x4", log(r1), "err", r1.chain_error())
r4 = mk()
r4.run(batches)
print("run4  ", log(r4), "err", r4.chain_error())
same = [pool[0]] * 4
ch2 = mk()
for c in same:
    ch2.step(controls=c)
ch2.flush()
print("chain same", log(ch2))
r5 = mk()
r5.run(same)
print("run same  ", log(r5), "err", r5.chain_error())

import time  # noqa: E402
pool8 = [eng.sample_controls(V, B, n, ns, 500 + i) for i in range(8)]
for K in (8, 16, 32, 64, 130):
    b = [pool8[i % 8] for i in range(K)]
    c = mk()
    for x in b:
        c.step(controls=x)
    c.flush()
    want = log(c)
    r = mk()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r.run(b)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    err = r.chain_error()
    got = log(r)
    bad = [i for i, (g, w) in enumerate(zip(got, want)) if g != w]
    print(f"K={K} run {dt * 1e3:.2f} ms err {err} first-bad {bad[:5]} n={len(got)}/{len(want)}")
    if bad:
        i = bad[0]
        print("  got ", got[max(0, i - 1):i + 2])
        print("  want", want[max(0, i - 1):i + 2])
