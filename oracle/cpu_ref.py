"""Reference-structured Python CPU path, used as bench.py's cpu_baseline.

TEST/BENCH INFRASTRUCTURE ONLY (kind "port"): a restatement of the
reference's per-candidate loop as it runs in CPython — every integral is a
`scipy.integrate.quad` call on a Python integrand, exactly like
integrate_velocity / integrate_angle (math_model_tree.py:91-96), and the
step / cost follow iteration_of_predict (:111-115) and control_criterion
(:82-87).  The reference itself cannot travel to the GPU box, so this port is
what gets timed there; it is validated bitwise against the reference's own
outputs in tests/test_cpu_ref.py.

Only the expansion is timed (the reference timer :307 -> :362 semantics):
the CoordinateTree's S1^3 object allocation is not reproduced for sampled
candidate sets (it is infeasible beyond ~5e3 candidates).
"""
import math
import os
import time

import numpy as np
import scipy.integrate as sp

L = 0.5
DELTA_T = 0.05


def _v_x(time_, velocity, phi):
    return velocity * np.cos(phi)


def _v_y(time_, velocity, phi):
    return velocity * np.sin(phi)


def _v_phi(time_, velocity, beta):
    return (velocity / L) * math.tan(beta)


def step(state, v, beta, t):
    dphi = sp.quad(_v_phi, t, t + DELTA_T, args=(v, beta))[0]
    ph = state[2] + dphi
    dx = sp.quad(_v_x, t, t + DELTA_T, args=(v, ph))[0]
    dy = sp.quad(_v_y, t, t + DELTA_T, args=(v, ph))[0]
    return [state[0] + dx, state[1] + dy, ph]


def cost(x, y, x_t, y_t, x_0, y_0):
    dist_t = math.sqrt((x_t - x) ** 2 + (y_t - y) ** 2)
    if x == x_0 and y == y_0:
        d = 1000
    else:
        d = (abs((y_t - y_0) * x - (x_t - x_0) * y + x_t * y_0 - y_t * x_0)
             / math.sqrt((y_t - y_0) ** 2 + (x_t - x_0) ** 2))
    return 10000 * dist_t + 10000 * d ** 2


def expand(problem, v_sc, b_sc, lo, hi, incumbent=math.inf):
    """Strict-< scan over candidates [lo, hi) (math_model_tree.py:337-360)."""
    x, y, phi, x_t, y_t, x_0, y_0, _L, t_a, _t_b = problem
    best, winner = incumbent, -1
    n_steps = len(v_sc)
    for c in range(lo, hi):
        s = [x, y, phi]
        for k in range(n_steps):
            s = step(s, float(v_sc[k][c]), float(b_sc[k][c]), t_a)
        cc = cost(s[0], s[1], x_t, y_t, x_0, y_0)
        if cc < best:
            best, winner = cc, c
    return best, winner


def _timed_worker(args):
    problem, v_sc, b_sc, lo, hi, budget_s = args
    t0 = time.perf_counter()
    done = lo
    best = (math.inf, -1)
    chunk = 16
    while done < hi and time.perf_counter() - t0 < budget_s:
        b = expand(problem, v_sc, b_sc, done, min(hi, done + chunk))
        best = min(best, b)
        done = min(hi, done + chunk)
    return done - lo, time.perf_counter() - t0, best


def granted_cores():
    """The host cores this process may use: its CPU affinity, bounded by the
    cgroup's CPU quota when one is set (a GPU box's share of a large host
    shows the whole machine in its affinity mask; the quota is the grant).
    Returns (cores, evidence dict)."""
    affinity = len(os.sched_getaffinity(0))
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max",):                       # cgroup v2
        try:
            q, period = open(path).read().split()[:2]
            if q != "max":
                quota = float(q) / float(period)
        except (OSError, ValueError):
            pass
    if quota is None:                                              # cgroup v1
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            period = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / period
        except (OSError, ValueError):
            pass
    cores = affinity if quota is None else max(1, min(affinity, int(quota + 0.5)))
    return cores, {"affinity_cpus": affinity, "cgroup_cpu_quota": quota}


def timed_rate(problem, v_sc, b_sc, budget_s=10.0, cores=None, max_per_core=40_000):
    """Candidates/s of the port on `cores` processes (default: every core the
    host grants, granted_cores()), each scanning its own contiguous slice of
    the candidate set for ~budget_s seconds."""
    import multiprocessing as mp
    evidence = {}
    if cores is None:
        cores, evidence = granted_cores()
    v_sc, b_sc = np.asarray(v_sc), np.asarray(b_sc)
    n = v_sc.shape[1]
    per = max(1, n // cores)
    m = min(per, max_per_core)
    tasks = [(problem, v_sc[:, r * per:r * per + m].copy(), b_sc[:, r * per:r * per + m].copy(),
              0, m, budget_s) for r in range(cores)]
    t0 = time.perf_counter()
    if cores == 1:
        outs = [_timed_worker(tasks[0])]
    else:
        with mp.get_context("fork").Pool(cores) as pool:
            outs = pool.map(_timed_worker, tasks)
    wall = time.perf_counter() - t0
    done = sum(o[0] for o in outs)
    busy = max(o[1] for o in outs)
    return {"candidates": done, "wall_s": wall, "busy_s": busy, "cores": cores,
            "rate": done / busy, **evidence}
