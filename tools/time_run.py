"""Wall time per step of the persistent run (any library variant via
DIPLOMJOURNEY_MPC_LIB).  python tools/time_run.py [n] [ns] [K] [reps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from diplomjourney_amd import math_model_tree as mmt  # noqa: E402
from diplomjourney_amd.episode import DeviceEpisode  # noqa: E402
from diplomjourney_amd.expansion import Expansion  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    ns = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    eng = Expansion("cuda:0")
    V = torch.tensor(mmt.vector_of_velocities(0.5), dtype=torch.float64, device="cuda")
    B = torch.tensor(mmt.vector_of_beta_angles(0.0), dtype=torch.float64, device="cuda")
    pool = [eng.sample_controls(V, B, n, ns, 0x5EED0000 + i) for i in range(min(K, 60))]
    batches = [pool[i % len(pool)] for i in range(K)]
    ep = DeviceEpisode(eng, n, ns, integrator="rect+cum", log_capacity=8192)
    ep.run(batches[:20])
    ep._ptr_table(batches)
    out = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ep.run(batches)
        torch.cuda.synchronize()
        out.append((time.perf_counter() - t0) / K * 1e6)
    lib = os.environ.get("DIPLOMJOURNEY_MPC_LIB", "default")
    print(f"{os.path.basename(lib)} n={n} ns={ns} K={K}: us/step " +
          " ".join(f"{x:.1f}" for x in out) + f"  chain_error={ep.chain_error()}")


if __name__ == "__main__":
    main()
