"""CPU oracle of the full-tree MPC (run_math_model.py) against
fixtures produced by running the reference at a reduced grid
(tests/golden/make_golden_fulltree.py: S1 = 25, 15625 leaves per step)."""
import json
import math
import os

import numpy as np
import pytest

from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                    "fulltree_reference.json")


@pytest.fixture(scope="module")
def gold():
    with open(GOLD) as fh:
        return json.load(fh)


def window(t_pre, dt):
    t = t_pre + dt                      # predictive_control: t += delta_t (:156)
    return t, t + dt


def test_leaf_detail_bitwise(gold):
    """All 15625 leaf costs and states, and every layer-0 / layer-1 state of
    the first call equal the reference's bit for bit."""
    cfg, det = gold["config"], gold["detail"]
    ep = gold["episodes"][det["episode"]]
    call = ep["calls"][det["call"]]
    t_a, t_b = window(call["pre"]["t"], cfg["delta_t"])
    r = O.fulltree_argmin(gold["vector_v"], gold["vector_beta"],
                          (call["x"], call["y"], call["phi"]), (ep["x_t"], ep["y_t"]),
                          (ep["x_0"], ep["y_0"]), float(np.arctan(ep["x_t"] / ep["y_t"])),
                          cfg["L"], t_a, t_b, call["pre"]["optimal_criterion"], detail=True)
    assert det["S1"] == 25
    assert np.array_equal(r["costs"], np.array(det["leaf_costs"]))
    assert np.array_equal(r["leaf_states"], np.array(det["leaf_states_last_layer"]))
    assert np.array_equal(r["layer0"], np.array(det["layer0_states"]))
    assert np.array_equal(r["layer1"], np.array(det["layer1_states"]))


def test_episodes_replayed(gold):
    """Every recorded MPC step of the three reference episodes: the oracle's
    winner gives the same returned state/control and the same new incumbent
    (bitwise), including steps where no leaf beats the never-reset incumbent
    (the reference then returns its previous winner again)."""
    cfg = gold["config"]
    V, B = gold["vector_v"], gold["vector_beta"]
    nb = len(B)
    n_steps = 0
    for ep in gold["episodes"]:
        atan_t = float(np.arctan(ep["x_t"] / ep["y_t"]))
        assert math.isclose(ep["first_incumbent"],
                            O.fulltree_cost(ep["x_0"], ep["y_0"], ep["phi_0"], ep["x_t"],
                                            ep["y_t"], ep["x_0"], ep["y_0"], atan_t),
                            rel_tol=0, abs_tol=0)
        prev = None
        for call in ep["calls"]:
            t_a, t_b = window(call["pre"]["t"], cfg["delta_t"])
            r = O.fulltree_argmin(V, B, (call["x"], call["y"], call["phi"]),
                                  (ep["x_t"], ep["y_t"]), (ep["x_0"], ep["y_0"]), atan_t,
                                  cfg["L"], t_a, t_b, call["pre"]["optimal_criterion"])
            if r["found"]:
                k0 = r["leaf"] // (len(V) * nb) ** 2
                ret = r["traj"][0] + [V[k0 // nb], B[k0 % nb]]
                crit = r["cost"]
            else:
                ret, crit = prev, call["pre"]["optimal_criterion"]
            assert ret == call["ret"]
            assert crit == call["post"]["optimal_criterion"]
            prev = ret
            n_steps += 1
    assert n_steps == 10
