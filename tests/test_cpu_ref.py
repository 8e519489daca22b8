"""The Python CPU port timed as bench.py's cpu_baseline reproduces the
reference bit for bit (it uses scipy.integrate.quad exactly as the reference
does, math_model_tree.py:91-115)."""
import numpy as np

from conftest import call_controls, call_problem
from oracle import cpu_ref


def test_port_step_bitwise(units):
    for r in units["steps"][:500]:
        x, y, phi, v, b, t = r["in"]
        assert [float(z) for z in cpu_ref.step([x, y, phi], v, b, t)] == r["out"]


def test_port_cost_bitwise(units):
    for r in units["costs"][:500]:
        xt, yt, x0, y0, px, py = r["in"]
        assert cpu_ref.cost(px, py, xt, yt, x0, y0) == r["cost"]


def test_port_scan_matches_reference(scenario):
    for rec in scenario["calls"][:40]:
        v_sc, b_sc = call_controls(rec)
        best, winner = cpu_ref.expand(call_problem(rec).as_tuple(), v_sc, b_sc, 0,
                                      v_sc.shape[1], rec["pre"]["optimal_criterion"])
        B = len(rec["B"])
        assert (v_sc[0][winner], rec["B"][winner % B]) == (rec["post"]["result_v"],
                                                          rec["post"]["result_beta"])


def test_timed_rate_runs():
    prob = (0.0, 0.0, 0.0, 2, 3, 0, 0, 0.5, 0.05, 0.1)
    v = np.full((3, 64), 0.5)
    b = np.linspace(-1, 1, 64)[None, :].repeat(3, 0)
    r = cpu_ref.timed_rate(prob, v, b, budget_s=0.2, cores=2)
    assert r["candidates"] > 0 and r["rate"] > 0 and r["cores"] == 2
