"""A/B of the chained step's launch knobs (MPC_CHAIN_BLOCKS, MPC_ANYORDER) at
config C: per variant, 300 warm + 200 timed chained launches (HIP events,
rotating over 8 resident batches), variants interleaved for R rounds.
Timing only (a variant's flush is not used).
    python tools/ab_chain.py [rounds] VAR=VAL,VAR=VAL ...   ("-" = defaults)"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from diplomjourney_amd import math_model_tree as mmt  # noqa: E402
from diplomjourney_amd.episode import DeviceEpisode  # noqa: E402
from diplomjourney_amd.expansion import Expansion  # noqa: E402


def main():
    rounds = int(sys.argv[1])
    variants = sys.argv[2:]
    n = int(os.environ.get("AB_N", "1000000"))
    ns = int(os.environ.get("AB_NS", "10"))
    eng = Expansion("cuda:0")
    V = torch.tensor(mmt.vector_of_velocities(0.5), dtype=torch.float64, device="cuda")
    B = torch.tensor(mmt.vector_of_beta_angles(0.0), dtype=torch.float64, device="cuda")
    pool = [eng.sample_controls(V, B, n, ns, 0x5EED0000 + i) for i in range(8)]
    res = {v: [] for v in variants}
    for _ in range(rounds):
        for var in variants:
            for k in ("MPC_CHAIN_BLOCKS", "MPC_ANYORDER"):
                os.environ.pop(k, None)
            if var != "-":
                for kv in var.split(","):
                    k, val = kv.split("=")
                    os.environ[k] = val
            ep = DeviceEpisode(eng, n, ns, integrator="rect+cum", chain=True, log_capacity=8192)
            for i in range(300):
                ep.step(controls=pool[i % 8])
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(200):
                ep.step(controls=pool[(i + 3) % 8])
            e1.record()
            torch.cuda.synchronize()
            res[var].append(e0.elapsed_time(e1) / 200 * 1e3)
            ep._pending = None
            del ep
    for var, xs in res.items():
        print(f"{var:40s} " + " ".join(f"{x:6.2f}" for x in xs) + f"   min {min(xs):6.2f} us",
              flush=True)


if __name__ == "__main__":
    main()
