"""A/B timing of the rollout kernel alone (developer tool, not the product):
rotate over NB distinct HBM-resident batches (NB x batch >> 256 MiB Infinity
Cache), time REPS launches between HIP events on the launch stream.
    DIPLOMJOURNEY_MPC_LIB=tools/var_x.so python tools/ab_kernel.py [n] [steps] [integ]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from diplomjourney_amd import math_model_tree as mmt  # noqa: E402
from diplomjourney_amd.abi import make_problem  # noqa: E402
from diplomjourney_amd.expansion import Expansion  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    ns = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    integ = sys.argv[3] if len(sys.argv) > 3 else "rect+rot"
    reps, nb = 40, 8
    eng = Expansion("cuda:0")
    V = torch.tensor(mmt.vector_of_velocities(0.5), dtype=torch.float64, device="cuda")
    B = torch.tensor(mmt.vector_of_beta_angles(0.0), dtype=torch.float64, device="cuda")
    pool = [eng.sample_controls(V, B, n, ns, 7 + i) for i in range(nb)]
    prob = make_problem(0.0, 0.0, 0.3, 2, 3, 0, 0, 0.5, 0.05, 0.1)
    for i in range(nb):
        eng.partials(prob, *pool[i], integ)
    torch.cuda.synchronize()
    out = {"lib": os.path.basename(os.environ.get("DIPLOMJOURNEY_MPC_LIB", "in-tree")),
           "n": n, "steps": ns, "integ": integ}
    for name, sel in (("hbm", lambda i: pool[i % nb]), ("cached", lambda i: pool[0])):
        passes = []
        for _ in range(5):      # median of 5 passes: one slow pass does not decide an A/B
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(reps):
                eng.partials(prob, *sel(i), integ)
            e1.record()
            torch.cuda.synchronize()
            passes.append(e0.elapsed_time(e1) / reps * 1e3)
        us = sorted(passes)[2]
        out[name + "_us"] = round(us, 2)
        out[name + "_min_us"] = round(min(passes), 2)
        out[name + "_TBs"] = round(16 * ns * n / us / 1e6, 3)
    r = eng.fetch(eng.rollout_argmin(prob, *pool[0], incumbent=1e300, integrator=integ))
    out["index"] = r.index
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
