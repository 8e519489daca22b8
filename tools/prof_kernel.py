"""Minimal driver for rocprofv3 counter passes: sample one candidate set,
then launch only the rollout kernel `reps` times.
    python tools/prof_kernel.py [n_cand] [n_steps] [integ] [reps]"""
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
    integ = sys.argv[3] if len(sys.argv) > 3 else "rect"
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
    eng = Expansion("cuda:0")
    V = torch.tensor(mmt.vector_of_velocities(0.5), dtype=torch.float64, device="cuda")
    B = torch.tensor(mmt.vector_of_beta_angles(0.0), dtype=torch.float64, device="cuda")
    v, b = eng.sample_controls(V, B, n, ns, 7)
    prob = make_problem(0.0, 0.0, 0.3, 2, 3, 0, 0, 0.5, 0.05, 0.1)
    for _ in range(reps):
        eng.partials(prob, v, b, integ)
    torch.cuda.synchronize()
    print("done", n, ns, integ, reps)


if __name__ == "__main__":
    main()
