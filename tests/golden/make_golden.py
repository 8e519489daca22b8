#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ by RUNNING THE REFERENCE.

Container-only test infrastructure: this script reads ``/root/reference`` at run
time (that tree does not exist on the GPU box) and is never imported by the
product, by ``bench.py`` or by ``smoke()``.  Only its *outputs* (JSON data:
inputs and expected outputs) are committed; no reference source is copied.

How the reference is executed:

* an environment shim reproduces the 2018 numpy/scipy star-import surface that
  ``math_model_tree.py:11`` relies on (``cos, sin, tan, arctan, size, math,
  random`` re-exported from scipy; ``random`` is numpy.random, as it was then),
  maps ``np.set_printoptions(threshold=np.nan)`` (``math_model_tree.py:17``) to
  ``sys.maxsize`` and makes matplotlib headless.  No reference logic changes.
* ``math_model_tree.py`` is read as text, split at its ``MODELLING`` marker
  (``math_model_tree.py:732-734``); the head is exec'd into a namespace, the
  namespace's ``predictive_control`` (``:278``) and ``new_target`` (``:118``)
  are wrapped by recorders, then the tail (``:736-738``: the model run and the
  "actual" run) is exec'd.  ``np.random.seed(0)`` is set before the actual run
  (its perturbations ``:259-275`` draw from numpy's global RNG).

Outputs:
  reference_scenario.json   every predictive_control call (inputs, globals,
                            outputs), operator events, episode trajectories
  reference_candidates.json per-candidate layer states + costs for 6 calls
  reference_units.json      unit vectors: kinematic step, cost, grids,
                            CoordinateTree index arithmetic, is_on_target

Run:  python tests/golden/make_golden.py      (≈90 s, one core)
"""
import contextlib
import io
import json
import math
import os
import random as pyrandom
import sys
import time

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def install_shim():
    import numpy as np
    import scipy
    import matplotlib

    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    plt.show = lambda *a, **k: None
    orig = np.set_printoptions

    def set_printoptions(*a, **k):
        thr = k.get("threshold")
        if isinstance(thr, float) and math.isnan(thr):
            k["threshold"] = sys.maxsize
        return orig(*a, **k)

    np.set_printoptions = set_printoptions
    extra = dict(cos=np.cos, sin=np.sin, tan=np.tan, arctan=np.arctan,
                 size=np.size, math=math, random=np.random)
    for name, obj in extra.items():
        setattr(scipy, name, obj)
        if name not in scipy.__all__:
            scipy.__all__.append(name)


def f(x):
    """Python/numpy scalar -> JSON value (floats stay exact via repr)."""
    if isinstance(x, bool):
        return x
    if isinstance(x, int):
        return x
    try:
        import numpy as np
        if isinstance(x, np.integer):
            return int(x)
    except ImportError:
        pass
    return float(x)


def fl(xs):
    return [f(x) for x in xs]


def load_reference():
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    install_shim()
    sys.path.insert(0, REF)
    src = open(os.path.join(REF, "math_model_tree.py")).read()
    marker = '"""\nMODELLING\n"""'
    assert src.count(marker) == 1
    head, tail = src.split(marker)
    ns = {"__name__": "reference_math_model_tree"}
    with contextlib.redirect_stdout(io.StringIO()):
        exec(compile(head, os.path.join(REF, "math_model_tree.py"), "exec"), ns)
    return ns, tail


GLOBALS = ("t", "x_t", "y_t", "x_0", "y_0", "steps_for_slowing",
           "optimal_criterion", "m", "result_v", "result_beta")


def per_candidate(ns, rec):
    """Per-candidate layer states and costs using the reference's own
    iteration_of_predict / control_criterion (math_model_tree.py:111,82),
    enumerated like predictive_control (:308-350)."""
    import numpy as np
    V, B = rec["V"], rec["B"]
    sfs = rec["pre"]["steps_for_slowing"]
    s0 = [rec["x"], rec["y"], rec["phi"]]
    layers = [[], [], []]
    costs = []
    for vel in V:
        if sfs > 0:
            vel = np.min(V) if np.min(V) > ns["v_min"] else ns["v_min"]
        for ang in B:
            s = s0
            for i in range(3):
                s = ns["iteration_of_predict"](s, vel, ang)
                layers[i].append(fl(s[:3]))
            costs.append(f(ns["control_criterion"](s)))
    return {"call": rec["call"], "layers": layers, "costs": costs}


def main():
    t0 = time.time()
    ns, tail = load_reference()
    import numpy as np

    calls, events = [], []
    cand_detail = []
    want_detail = {0, 1, 59, 150}
    slow_seen = {False: False, True: False}
    orig_pc = ns["predictive_control"]
    orig_nt = ns["new_target"]
    orig_mpc = ns["math_mpc"]

    def pc(x, y, phi, tx, ty, V, B, isActual):
        i = len(calls)
        pre = {k: f(ns[k]) for k in GLOBALS}
        prev_traj = ns["optimal_trajectory"][0]
        ret = orig_pc(x, y, phi, tx, ty, V, B, isActual)
        traj = ns["optimal_trajectory"][0]
        rec = {
            "call": i, "isActual": bool(isActual),
            "x": f(x), "y": f(y), "phi": f(phi), "target_x": f(tx), "target_y": f(ty),
            "V": fl(V), "B": fl(B), "pre": pre,
            "post": {k: f(ns[k]) for k in GLOBALS},
            "found": traj is not prev_traj,
            "traj": [fl(s) for s in traj],
            "ret": fl(ret),
        }
        calls.append(rec)
        slow = pre["steps_for_slowing"] > 0
        if i in want_detail or (slow and not slow_seen[bool(isActual)]):
            if slow:
                slow_seen[bool(isActual)] = True
            cand_detail.append(per_candidate(ns, rec))
        return ret

    def nt(ax, ay, aphi, tx, ty, av):
        pre = {k: f(ns[k]) for k in GLOBALS}
        orig_nt(ax, ay, aphi, tx, ty, av)
        events.append({"after_call": len(calls) - 1, "p": f(ns.get("p", 0)),
                       "args": fl([ax, ay, aphi, tx, ty, av]), "pre": pre,
                       "post": {k: f(ns[k]) for k in GLOBALS}})

    def mpc(initial, target, isActual):
        if isActual:
            np.random.seed(0)
        return orig_mpc(initial, target, isActual)

    ns["predictive_control"] = pc
    ns["new_target"] = nt
    ns["math_mpc"] = mpc
    # Only the two math_mpc calls of the tail are needed; the plotting after
    # them (:740-883) is skipped to keep matplotlib out of the fixture run.
    runs = tail.split("# ---------------------------------------------------------------")[1]
    with contextlib.redirect_stdout(io.StringIO()):
        exec(compile(runs, "math_model_tree.py<tail>", "exec"), ns)

    traj_names = ["result_trajectory_x", "result_trajectory_y", "result_trajectory_phi",
                  "result_trajectory_v", "result_trajectory_beta",
                  "actual_result_trajectory_x", "actual_result_trajectory_y",
                  "actual_result_trajectory_phi", "actual_result_trajectory_v",
                  "actual_result_trajectory_beta", "time_arr_for_plotting",
                  "actual_time_arr_for_plotting"]
    scenario = {
        "source": "math_model_tree.py:736-738 run under the SURVEY Appendix A shim; "
                  "np.random.seed(0) before the actual run",
        "first_incumbent": calls[0]["pre"]["optimal_criterion"],
        "calls": calls, "events": events,
        "trajectories": {k: fl(ns[k]) for k in traj_names},
    }
    with open(os.path.join(OUT, "reference_scenario.json"), "w") as fh:
        json.dump(scenario, fh, separators=(",", ":"))
    with open(os.path.join(OUT, "reference_candidates.json"), "w") as fh:
        json.dump({"calls": cand_detail}, fh, separators=(",", ":"))

    # ---------------- unit vectors ----------------
    rng = pyrandom.Random(20261015)
    saved = {k: ns[k] for k in GLOBALS}
    steps = []
    tvals = [0.0, 0.05, 0.1, 2.9499999999999975, 7.499999999999981]
    tacc = 0.0
    for _ in range(200):
        tacc += 0.05
    tvals.append(tacc)
    for k in range(3000):
        x, y = rng.uniform(-10, 10), rng.uniform(-10, 10)
        phi = rng.uniform(-math.pi, math.pi) * (3 if k % 7 == 0 else 1)
        v = rng.uniform(0, 1) if k % 3 else round(rng.randrange(0, 200) * 0.005, 12)
        b = rng.uniform(-1.06, 1.06) if k % 5 else rng.randrange(-60, 61) * ns["delta_beta"]
        t = rng.choice(tvals) if k % 2 else rng.uniform(0, 20)
        ns["t"] = t
        out = ns["iteration_of_predict"]([x, y, phi], v, b)
        steps.append({"in": [x, y, phi, v, b, t], "out": fl(out[:3])})
    costs = []
    for k in range(2000):
        xt, yt = (rng.randint(-10, 10), rng.randint(-10, 10)) if k % 4 == 0 else \
            (rng.uniform(-10, 10), rng.uniform(-10, 10))
        x0, y0 = (rng.randint(-10, 10), rng.randint(-10, 10)) if k % 4 == 1 else \
            (rng.uniform(-10, 10), rng.uniform(-10, 10))
        if (xt, yt) == (x0, y0):
            xt += 1
        if k % 10 == 3:
            px, py = x0, y0          # exact line-origin hit -> D = 1000
        else:
            px, py = rng.uniform(-10, 10), rng.uniform(-10, 10)
        ns["x_t"], ns["y_t"], ns["x_0"], ns["y_0"] = xt, yt, x0, y0
        c = ns["control_criterion"]([px, py, 0.0])
        costs.append({"in": [f(xt), f(yt), f(x0), f(y0), px, py], "cost": f(c)})
    for k, v in saved.items():
        ns[k] = v
    vin = [0, 0.0, 0.005, 0.2, 0.5, 0.99, 1.0, 0.9950000000000006, 0.025, 0.4, 0.97]
    vin += [rng.uniform(0, 1) for _ in range(20)]
    bin_ = [0, 0.0, 0.5, -0.5, ns["beta_max"], -ns["beta_max"], ns["beta_max"] + 0.001,
            0.3490658503988659, -7.632783294297951e-17]
    bin_ += [rng.uniform(-1.1, 1.1) for _ in range(20)]
    grids = {
        "velocities": [{"in": f(v), "out": fl(ns["vector_of_velocities"](v))} for v in vin],
        "betas": [{"in": f(b), "out": fl(ns["vector_of_beta_angles"](b))} for b in bin_],
    }
    CT = ns["CoordinateTree"]
    tree = []
    for s1 in (1, 2, 3, 4, 7):
        ct = CT(s1)
        tree.append({"S1": s1, "size": ct.get_size(),
                     "parents": [ct.get_index_of_parent(j) for j in range(ct.get_size())]})
    ct = CT(20)
    js = sorted({0, 19, 20, 21, 419, 420, 421, 8419, 8420} |
                {rng.randrange(0, ct.get_size()) for _ in range(200)})
    tree.append({"S1": 20, "size": ct.get_size(), "js": js,
                 "parents_at": [ct.get_index_of_parent(j) for j in js]})
    tree.append({"S1": 451, "size_formula": 451 + 451 ** 2 + 451 ** 3})
    ot = []
    for k in range(500):
        ax, ay = rng.uniform(-1, 3), rng.uniform(-1, 4)
        tx, ty = 2, 3
        if k % 5 == 0:
            ax, ay = tx + rng.uniform(-0.03, 0.03), ty + rng.uniform(-0.03, 0.03)
        r = ns["is_on_target"](ax, ay, tx, ty)
        ot.append({"in": [ax, ay, tx, ty], "out": [bool(r[0]), f(r[1])]})
    consts = {k: f(ns[k]) for k in ("L", "delta_t", "beta_max", "delta_beta", "beta_acc_max",
                                     "v_max", "v_min", "delta_v", "v_acc_max", "eps",
                                     "eps_beta", "phi_0", "radius_u_turn")}
    import config as ref_config  # /root/reference/config.py (container only)
    consts_cfg = {k: f(getattr(ref_config, k)) for k in dir(ref_config)
                  if not k.startswith("_") and k != "math"}
    units = {"steps": steps, "costs": costs, "grids": grids, "tree": tree,
             "is_on_target": ot, "consts_mmt": consts, "config": consts_cfg}
    with open(os.path.join(OUT, "reference_units.json"), "w") as fh:
        json.dump(units, fh, separators=(",", ":"))
    print(f"calls={len(calls)} events={len(events)} detail={len(cand_detail)} "
          f"steps={len(steps)} costs={len(costs)} in {time.time() - t0:.1f}s")


if __name__ == "__main__":
    main()
