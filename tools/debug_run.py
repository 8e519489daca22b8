"""Debug: persistent run vs the two-launch episode on one configuration;
prints the chain error, the first differing steps and the per-step
records' summary.  python tools/debug_run.py [n] [ns] [steps] [max_steps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from diplomjourney_amd import math_model_tree as mmt  # noqa: E402
from diplomjourney_amd.episode import DeviceEpisode  # noqa: E402
from diplomjourney_amd.expansion import Expansion  # noqa: E402


def log(ep):
    return [(r.step, r.index, r.cost, r.x, r.y, r.phi, r.p, r.episode) for r in ep.read_log()]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 50_000
    ns = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    eng = Expansion("cuda:0")
    V = torch.tensor(mmt.vector_of_velocities(0.5), dtype=torch.float64, device="cuda")
    B = torch.tensor(mmt.vector_of_beta_angles(0.0), dtype=torch.float64, device="cuda")
    pool = [eng.sample_controls(V, B, n, ns, 500 + i) for i in range(8)]
    batches = [pool[i % 8] for i in range(steps)]
    ref = DeviceEpisode(eng, n, ns, integrator="rect+cum", log_capacity=512)
    for c in batches:
        ref.step(controls=c)
    want = log(ref)
    ep = DeviceEpisode(eng, n, ns, integrator="rect+cum", log_capacity=512)
    ep.run(batches)
    got = log(ep)
    print("chain_error", ep.chain_error())
    bad = [i for i, (a, b) in enumerate(zip(got, want)) if a != b]
    print("differing steps", bad[:40], "of", len(want))
    for i in bad[:5]:
        print(" got ", got[i])
        print(" want", want[i])
    ws = ep._run_ws.cpu().numpy().view("uint64")
    T = -(-n // 512)
    base = 128 // 8 + 2 * 70
    for j in range(min(steps, 10)):
        half = ws[base + (j & 1) * T * 4: base + (j & 1) * T * 4 + T * 4].reshape(T, 4)
        tags = set(int(x) & 0xffffffff for x in half[:, :3].ravel())
        print("step", j, "half", j & 1, "tags", sorted(tags)[:6])


if __name__ == "__main__":
    main()
