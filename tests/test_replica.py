"""The kernel's arithmetic, built for the host (tests/replica_harness.cpp),
against the oracle (CPU) and against the GPU (bitwise).

* CPU: replica vs oracle — identical arg-min on reference-shaped inputs,
  states within a few ulp (the only difference is tan/sin/cos: device
  routines vs glibc, and x*x vs glibc pow(x, 2) in the cost).
* GPU: the kernel's states (CoordinateTree output) and its winner's cost are
  the replica's BIT FOR BIT — the device code does exactly the IEEE
  operations it was written to do.  The one non-IEEE instruction, the
  steering tangent's reciprocal estimate (v_rcp_f64), is supplied to the
  replica from the device (harness.replica_rollout(device_estimates=True)).
"""
import sys

import numpy as np
import pytest
import torch

from conftest import call_controls, call_problem
from harness import replica_rollout

INC_MAX = float(sys.maxsize)


def _case(n, ns, seed):
    from oracle import oracle as O
    from diplomjourney_amd import math_model_tree as mmt
    V = mmt.vector_of_velocities(0.5)
    B = mmt.vector_of_beta_angles(0.0)
    return O.sample_controls(V, B, n, ns, seed)


def test_replica_vs_oracle_scenario(scenario, oracle):
    for rec in scenario["calls"][::7]:
        v, b = call_controls(rec)
        for integ in ("qk21", "rect"):
            st, costs = replica_rollout(call_problem(rec), v, b, integ)
            ref, rc, rs = oracle.rollout_argmin(call_problem(rec), v, b, integ=integ,
                                                want_costs=True, want_states=True)
            assert int(np.argmin(costs)) == ref.index
            assert np.abs(st - rs).max() <= 1e-15
            assert np.allclose(costs, rc, rtol=1e-14, atol=0)


def test_replica_vs_oracle_synthetic(oracle):
    from diplomjourney_amd.abi import make_problem
    v, b = _case(20_000, 10, 5)
    p = make_problem(0.2, -0.1, 2.9, 2, 3, 0.5, 0.5, 0.5, 0.35, 0.4)
    st, costs = replica_rollout(p, v, b, "rect")
    ref, rc, rs = oracle.rollout_argmin(p, v, b, integ="rect", want_costs=True, want_states=True)
    assert int(np.argmin(costs)) == ref.index
    assert np.abs(st - rs).max() <= 1e-14
    frac_equal = np.mean(st == rs)
    assert frac_equal > 0.5                 # most states bit-identical to the reference math


@pytest.mark.parametrize("integ", ["rect+rot", "rect+cum"])
def test_replica_rotation_mode_vs_oracle(oracle, integ):
    """Heading-rotation modes (rotation of the pose's heading; rotation from
    the identity with the pose applied last): a few ulp from the reference's
    direct sin/cos, same arg-min."""
    from diplomjourney_amd.abi import make_problem
    v, b = _case(20_000, 12, 6)
    p = make_problem(0.2, -0.1, 2.9, 2, 3, 0.5, 0.5, 0.5, 0.35, 0.4)
    st, costs = replica_rollout(p, v, b, integ)
    ref, rc, rs = oracle.rollout_argmin(p, v, b, integ="rect", want_costs=True, want_states=True)
    assert int(np.argmin(costs)) == ref.index
    assert np.abs(st - rs).max() <= 1e-13
    assert np.allclose(costs, rc, rtol=1e-13, atol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("n,ns,integ", [(100_000, 5, "rect"), (30_001, 12, "qk21"),
                                        (4096, 32, "rect"), (100_000, 10, "rect+rot"),
                                        (30_001, 7, "qk21+rot"), (100_000, 10, "rect+cum"),
                                        (30_001, 9, "rect+cum")])
def test_gpu_bitwise_equals_replica(engine, n, ns, integ):
    from diplomjourney_amd.abi import make_problem
    v, b = _case(n, ns, 11)
    p = make_problem(-1.0, 0.5, -2.2, 2, 3, 0.25, -0.5, 0.5, 7.45, 7.5)
    st, costs = replica_rollout(p, v, b, integ, device_estimates=True)
    vd = torch.as_tensor(v, device="cuda")
    bd = torch.as_tensor(b, device="cuda")
    states = torch.empty((ns, 3, n), dtype=torch.float64, device="cuda")
    engine.rollout_argmin(p, vd, bd, incumbent=INC_MAX, integrator=integ, states=states)
    got = engine.fetch()
    assert np.array_equal(states.cpu().numpy(), st)
    k = int(np.argmin(costs))
    assert got.index == k and got.cost == costs[k]
    engine.rollout_argmin(p, vd, bd, incumbent=INC_MAX, integrator=integ)   # streaming path
    fast = engine.fetch()
    assert fast.index == k and fast.cost == costs[k]
    assert fast.trajectory() == [list(st[s, :, k]) for s in range(ns)]


@pytest.mark.gpu
@pytest.mark.parametrize("integ", ["rect", "rect+rot"])
def test_gpu_trig_bitwise_equals_host_build(engine, integ):
    """The device build of mpc_trig.h (device rint/fma; tan_small's hardware
    reciprocal estimates handed to the host build) against its host build, through the
    production kernel: every state of 2e6 candidates with uniformly random
    steering angles over the whole regular range |beta| <= 1.1 (not just the
    reference grid's 41 values) and random speeds, from a random start
    heading — bit for bit."""
    from diplomjourney_amd.abi import make_problem
    rng = np.random.default_rng(29)
    n, ns = 2_000_000, 2
    v = rng.uniform(0.0, 1.0, (ns, n))
    b = rng.uniform(-1.1, 1.1, (ns, n))
    p = make_problem(0.3, -0.7, rng.uniform(-3, 3), 2, 3, 0, 0, 0.5, 0.05, 0.1)
    st, costs = replica_rollout(p, v, b, integ, device_estimates=True)
    states = torch.empty((ns, 3, n), dtype=torch.float64, device="cuda")
    engine.rollout_argmin(p, torch.as_tensor(v, device="cuda"), torch.as_tensor(b, device="cuda"),
                          incumbent=INC_MAX, integrator=integ, states=states)
    got = states.cpu().numpy()
    assert np.array_equal(got, st), int((got != st).sum())
    assert engine.fetch().cost == costs.min()


@pytest.mark.gpu
@pytest.mark.parametrize("integ", ["rect+rot", "rect", "qk21", "qk21+rot", "rect+cum"])
def test_gpu_irregular_candidates_stream_kernel(engine, integ):
    """Irregular candidates (|beta| > 1.1 at some step; in rotation mode also
    |dphi| > 0.2) leave the streaming kernel's fast loop and are recomputed
    with the safe recurrence (full-range trig) in the same lane.  Winner,
    cost and trajectory equal the host replica bit for bit: (a) most
    candidates irregular, irregular winner; (b) a few irregular candidates
    scattered over otherwise regular blocks; (c) 2.1e6 candidates, so blocks
    stride over several tiles, with irregular candidates only in late tiles;
    (d) huge arguments (Payne-Hanek reduction on the device)."""
    from diplomjourney_amd.abi import make_problem
    rng = np.random.default_rng(3)
    p = make_problem(0, 0, 0, 0.3, 0.8, 0, 0, 0.5, 0.05, 0.1)
    cases = []
    n, ns = 200_000, 10
    cases.append((rng.uniform(0, 1, (ns, n)), rng.uniform(-1.25, 1.25, (ns, n)), True))
    v, b = _case(n, ns, 12)
    hit = rng.choice(n, 40, replace=False)
    b[rng.integers(0, ns, 40), hit] = 1.2
    cases.append((v, b, None))
    n = 2 * 2048 * 512 + 1000
    v, b = _case(n, 4, 13)
    b[2, [2048 * 512 + 7, n - 3, n - 600]] = -1.15
    cases.append((v, b, None))
    # (d) huge steering angles and headings: the safe recurrence's trig takes
    # the Payne-Hanek reduction (mpc_trig.h reduce_pio2_large) on the device,
    # bit for bit the host's
    n, ns = 50_000, 6
    v, b = _case(n, ns, 14)
    hit = rng.choice(n, 64, replace=False)
    b[1, hit[:32]] = rng.uniform(1e6, 1e300, 32) * rng.choice([-1, 1], 32)
    v[3, hit[32:]] = rng.uniform(1e7, 1e12, 32)        # dphi and the heading become huge
    cases.append((v, b, None))
    for v, b, want_irregular in cases:
        st, costs = replica_rollout(p, v, b, integ, device_estimates=True)
        k = int(np.argmin(costs))
        if want_irregular:
            assert np.abs(b[:, k]).max() > 1.1       # the case exercises an irregular winner
        engine.rollout_argmin(p, torch.as_tensor(v, device="cuda"),
                              torch.as_tensor(b, device="cuda"), incumbent=INC_MAX,
                              integrator=integ)
        got = engine.fetch()
        assert got.index == k and got.cost == costs[k]
        assert got.trajectory() == [list(st[s, :, k]) for s in range(v.shape[0])]
