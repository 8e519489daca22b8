"""The CPU oracle (oracle/mpc_oracle.c) pinned against vectors produced by
running the reference itself (tests/golden/make_golden.py).

Bar: bitwise.  The oracle is the checker every GPU parity test uses, so it
must reproduce math_model_tree.py's arithmetic exactly first.
"""
import numpy as np

from conftest import call_controls, call_problem


def test_step_bitwise(units, oracle):
    """iteration_of_predict (math_model_tree.py:111-115) incl. sp.quad -> qk21."""
    bad = []
    for r in units["steps"]:
        x, y, phi, v, b, t = r["in"]
        out = oracle.step([x, y, phi], v, b, 0.5, t, t + 0.05, "qk21")
        if out != r["out"]:
            bad.append((r, out))
    assert not bad, f"{len(bad)} of {len(units['steps'])} steps differ, first {bad[0]}"


def test_cost_bitwise(units, oracle):
    """control_criterion (:82-87) incl. the line-origin sentinel and int globals."""
    n_origin = 0
    for r in units["costs"]:
        xt, yt, x0, y0, px, py = r["in"]
        n_origin += (px, py) == (x0, y0)
        assert oracle.cost(px, py, xt, yt, x0, y0) == r["cost"], r
    assert n_origin >= 100  # the D = 1000 branch is exercised


def test_qk21_is_not_plain_product(units, oracle):
    """qk21 on a constant differs from f*h in the last bits often enough that
    the restatement must keep it (SURVEY Fact 4)."""
    diff = sum(oracle.qk21(f, 1.0, 1.05) != f * (1.05 - 1.0)
               for f in np.linspace(-2, 2, 1001))
    assert diff > 0


def test_scenario_calls_bitwise(scenario, oracle):
    """All 349 predictive_control calls of math_model_tree.py:736-738:
    chosen (v, beta) and the 3 predicted states, bit for bit."""
    assert len(scenario["calls"]) == 349
    for rec in scenario["calls"]:
        v_sc, b_sc = call_controls(rec)
        res, _, _ = oracle.rollout_argmin(call_problem(rec), v_sc, b_sc,
                                          incumbent=rec["pre"]["optimal_criterion"],
                                          integ="qk21")
        assert res.found == rec["found"]
        assert (res.v, res.beta) == (rec["post"]["result_v"], rec["post"]["result_beta"])
        assert res.trajectory() == [s[:3] for s in rec["traj"]], rec["call"]


def test_scenario_calls_rect_same_choice(scenario, oracle):
    """The exact integral f*h selects the same control on every call, states
    within 1e-15 (SURVEY Fact 4: max 4.4e-16)."""
    worst = 0.0
    for rec in scenario["calls"]:
        v_sc, b_sc = call_controls(rec)
        res, _, _ = oracle.rollout_argmin(call_problem(rec), v_sc, b_sc,
                                          incumbent=rec["pre"]["optimal_criterion"],
                                          integ="rect")
        assert (res.v, res.beta) == (rec["post"]["result_v"], rec["post"]["result_beta"])
        for s, ref in zip(res.trajectory(), rec["traj"]):
            worst = max(worst, max(abs(a - b) for a, b in zip(s, ref[:3])))
    assert worst <= 1e-15


def test_candidate_layers_bitwise(scenario, candidates, oracle):
    """Per-candidate layer states and costs of 6 calls (incl. slow-down)."""
    calls = {r["call"]: r for r in scenario["calls"]}
    assert len(candidates["calls"]) == 6
    for det in candidates["calls"]:
        rec = calls[det["call"]]
        v_sc, b_sc = call_controls(rec)
        _, costs, states = oracle.rollout_argmin(call_problem(rec), v_sc, b_sc, integ="qk21",
                                                 want_costs=True, want_states=True)
        assert costs.tolist() == det["costs"]
        for layer in range(3):
            got = states[layer].T.tolist()
            assert got == det["layers"][layer]


def test_sampler_const_prefix_and_determinism(oracle):
    V = [0.1, 0.2, 0.3]
    B = [-0.5, 0.0, 0.5, 1.0]
    v1, b1 = oracle.sample_controls(V, B, 50, 4, seed=20261015)
    v2, b2 = oracle.sample_controls(V, B, 50, 4, seed=20261015)
    assert np.array_equal(v1, v2) and np.array_equal(b1, b2)
    for g in range(12):  # the reference's constant sequences first
        assert (v1[:, g] == V[g // 4]).all() and (b1[:, g] == B[g % 4]).all()
    v3, _ = oracle.sample_controls(V, B, 38, 4, seed=20261015, index_base=12)
    assert np.array_equal(v3, v1[:, 12:])  # sharding by index_base is consistent
    assert set(np.unique(v1)) <= set(V) and set(np.unique(b1)) <= set(B)
