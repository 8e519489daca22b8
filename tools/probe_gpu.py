"""Developer probe: parity spot-checks + kernel timings on one GPU.

Not part of the product or the test suite; prints one JSON object per check.
    python tools/probe_gpu.py [--quick]
"""
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from diplomjourney_amd import math_model_tree as mmt  # noqa: E402
from diplomjourney_amd.abi import make_problem  # noqa: E402
from diplomjourney_amd.expansion import Expansion  # noqa: E402
from oracle import oracle as O  # noqa: E402


def emit(**kw):
    print(json.dumps(kw), flush=True)


def grid_451():
    V = mmt.vector_of_velocities(0.5)
    B = mmt.vector_of_beta_angles(0.0)
    return V, B


def parity_synthetic(eng, n_cand, n_steps, integ, seed=20261015):
    V, B = grid_451()
    vg = torch.tensor(V, dtype=torch.float64, device="cuda")
    bg = torch.tensor(B, dtype=torch.float64, device="cuda")
    v_sc, b_sc = eng.sample_controls(vg, bg, n_cand, n_steps, seed)
    prob = make_problem(0.0, 0.0, 0.3, 2, 3, 0, 0, 0.5, 0.05, 0.1)
    eng.rollout_argmin(prob, v_sc, b_sc, incumbent=float(sys.maxsize), integrator=integ)
    got = eng.fetch()
    vh, bh = v_sc.cpu().numpy(), b_sc.cpu().numpy()
    ov, ob = O.sample_controls(V, B, n_cand, n_steps, seed)
    sampler_ok = bool(np.array_equal(vh, ov) and np.array_equal(bh, ob))
    t0 = time.time()
    ref, costs, _ = O.rollout_argmin(prob, vh, bh, incumbent=float(sys.maxsize), integ=integ,
                                     want_costs=True)
    t_oracle = time.time() - t0
    dtraj = max(abs(got.traj[s][k] - ref.traj[s][k]) for s in range(n_steps) for k in range(3))
    gap = abs(costs[got.index] - costs[ref.index]) / max(abs(costs[ref.index]), 1e-300)
    emit(check="synthetic", n_cand=n_cand, n_steps=n_steps, integ=integ, sampler_bitwise=sampler_ok,
         gpu_index=got.index, oracle_index=ref.index, same=got.index == ref.index,
         dtraj=dtraj, dcost_rel=abs(got.cost - ref.cost) / ref.cost, oracle_gap_rel=gap,
         oracle_s=round(t_oracle, 2))


def ulp_rate(eng, n_cand=200000):
    """How often do device fp64 tan/sincos differ from glibc (states after 1 step)?"""
    rng = np.random.default_rng(1)
    v = rng.uniform(0, 1, (1, n_cand))
    b = rng.uniform(-1.06, 1.06, (1, n_cand))
    prob = make_problem(0.0, 0.0, 0.0, 2, 3, 0, 0, 0.5, 0.05, 0.1)
    for phi0 in (0.0, 2.5):
        prob.phi = phi0
        vd = torch.tensor(v, device="cuda")
        bd = torch.tensor(b, device="cuda")
        states = torch.empty((1, 3, n_cand), dtype=torch.float64, device="cuda")
        eng.rollout_argmin(prob, vd, bd, integrator="rect", states=states)
        g = states.cpu().numpy()
        _, _, ref = O.rollout_argmin(prob, v, b, integ=1, want_states=True)
        neq = (g != ref).sum(axis=2)[0]
        emit(check="ulp_rate", phi0=phi0, n=n_cand, mismatch_x=int(neq[0]), mismatch_y=int(neq[1]),
             mismatch_phi=int(neq[2]), max_abs=float(np.abs(g - ref).max()))


def time_kernel(eng, n_cand, n_steps, integ, reps=20, odd=False):
    V, B = grid_451()
    vg = torch.tensor(V, dtype=torch.float64, device="cuda")
    bg = torch.tensor(B, dtype=torch.float64, device="cuda")
    n = n_cand - 1 if odd else n_cand
    v_sc, b_sc = eng.sample_controls(vg, bg, n, n_steps, 7)
    prob = make_problem(0.0, 0.0, 0.3, 2, 3, 0, 0, 0.5, 0.05, 0.1)
    for _ in range(3):
        eng.partials(prob, v_sc, b_sc, integ)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        eng.partials(prob, v_sc, b_sc, integ)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    gbs = 16.0 * n * n_steps / (ms * 1e-3) / 1e9
    emit(check="time", n_cand=n, n_steps=n_steps, integ=integ, cpl=1 if odd else 2, ms=round(ms, 4),
         rollouts_per_s=n / (ms * 1e-3), GBps=round(gbs, 1), frac_8TBs=round(gbs / 8000, 3))


def main():
    quick = "--quick" in sys.argv
    eng = Expansion("cuda:0")
    emit(check="device", name=torch.cuda.get_device_name(0),
         lib=os.environ.get("DIPLOMJOURNEY_MPC_LIB", "in-tree"))
    if "--time-only" in sys.argv:
        for n_steps, integ in ((10, "rect"), (10, "rect+rot"), (10, "qk21"), (10, "qk21+rot"),
                               (3, "rect"), (3, "rect+rot"), (12, "rect"), (12, "rect+rot")):
            time_kernel(eng, 1_000_000, n_steps, integ)
        time_kernel(eng, 8_000_000, 10, "rect")
        time_kernel(eng, 8_000_000, 10, "rect+rot")
        return
    for n_steps, integ in ((10, "rect"), (10, "qk21"), (3, "rect"), (12, "rect"), (11, "rect"), (8, "rect")):
        time_kernel(eng, 1_000_000, n_steps, integ)
    time_kernel(eng, 1_000_000, 10, "rect", odd=True)
    time_kernel(eng, 8_000_000, 10, "rect")
    ulp_rate(eng)
    parity_synthetic(eng, 100_000, 3, "qk21")
    parity_synthetic(eng, 100_000, 3, "rect")
    if not quick:
        parity_synthetic(eng, 1_000_000, 10, "rect")
        parity_synthetic(eng, 1_000_000, 10, "qk21")


if __name__ == "__main__":
    main()
