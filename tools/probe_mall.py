"""Developer probe: rollout kernel time on one repeated candidate batch vs a
rotation over distinct batches (Infinity-Cache residency), by-value vs
device-resident problem constants.  Prints one JSON object per case."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from diplomjourney_amd import math_model_tree as mmt  # noqa: E402
from diplomjourney_amd.abi import make_problem  # noqa: E402
from diplomjourney_amd.episode import DeviceEpisode  # noqa: E402
from diplomjourney_amd.expansion import Expansion  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    ns = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    integ = sys.argv[3] if len(sys.argv) > 3 else "rect+rot"
    eng = Expansion("cuda:0")
    V = torch.tensor(mmt.vector_of_velocities(0.5), dtype=torch.float64, device="cuda")
    B = torch.tensor(mmt.vector_of_beta_angles(0.0), dtype=torch.float64, device="cuda")
    pool = [eng.sample_controls(V, B, n, ns, 100 + i) for i in range(8)]
    prob = make_problem(0.0, 0.0, 0.3, 2, 3, 0, 0, 0.5, 0.05, 0.1)
    ep = DeviceEpisode(eng, n, ns, integrator=integ)
    reps = 24

    def run(label, fn):
        for i in range(4):
            fn(i)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(reps):
            fn(i)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / reps * 1e3
        print(json.dumps({"case": label, "n": n, "n_steps": ns, "integ": integ, "us": round(us, 2),
                          "frac_8TBs": round(16 * n * ns / (us * 1e-6) / 8e12, 3)}), flush=True)

    run("by-value, same batch", lambda i: eng.partials(prob, *pool[0], integ))
    run("by-value, 8 batches", lambda i: eng.partials(prob, *pool[i % 8], integ))

    def kdev(i, same):
        ep.cur = pool[0 if same else i % 8]
        ep.partials()
    run("device K, same batch", lambda i: kdev(i, True))
    run("device K, 8 batches", lambda i: kdev(i, False))


if __name__ == "__main__":
    main()
