"""Chained launches alone: REPS back-to-back mpc_episode_chain_step launches
between HIP events (any library variant via DIPLOMJOURNEY_MPC_LIB; results
are not checked — timing probe).  python tools/time_chain.py [n] [ns] [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from diplomjourney_amd import math_model_tree as mmt  # noqa: E402
from diplomjourney_amd.episode import DeviceEpisode  # noqa: E402
from diplomjourney_amd.expansion import Expansion  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    ns = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    eng = Expansion("cuda:0")
    V = torch.tensor(mmt.vector_of_velocities(0.5), dtype=torch.float64, device="cuda")
    B = torch.tensor(mmt.vector_of_beta_angles(0.0), dtype=torch.float64, device="cuda")
    pool = [eng.sample_controls(V, B, n, ns, 0x5EED0000 + i) for i in range(8)]
    ep = DeviceEpisode(eng, n, ns, integrator="rect+cum", chain=True, log_capacity=8192)
    for i in range(20):
        ep.step(controls=pool[i % 8])
    out = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for i in range(reps):
            ep.step(controls=pool[i % 8])
        e1.record()
        torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1) / reps * 1e3)
    ep.flush()
    torch.cuda.synchronize()
    lib = os.environ.get("DIPLOMJOURNEY_MPC_LIB", "in-tree")
    print(f"{os.path.basename(lib)} chained launch us: " + " ".join(f"{x:.2f}" for x in out))


if __name__ == "__main__":
    main()
