"""Full-tree MPC on the GPU (mpc_fulltree_argmin, csrc/mpc_fulltree.h) against
the CPU oracle and the reference fixtures (tests/golden/fulltree_reference.json)."""
import json
import math
import os

import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                    "fulltree_reference.json")
STATE_TOL = 1e-9
COST_RTOL = 1e-12


@pytest.fixture(scope="module")
def gold():
    with open(GOLD) as fh:
        return json.load(fh)


def _device_call(engine, V, B, state, target, origin, atan_t, L, t_a, t_b, inc, integ):
    from diplomjourney_amd.abi import MpcFulltreeProblem
    from diplomjourney_amd.expansion import fulltree_argmin, fulltree_result
    vg = torch.tensor(V, dtype=torch.float64, device=engine.device)
    bg = torch.tensor(B, dtype=torch.float64, device=engine.device)
    p = MpcFulltreeProblem(*state, *target, *origin, atan_t, L, t_a, t_b)
    return fulltree_result(fulltree_argmin(engine, p, vg, bg, inc, integ))


def _agree(dev, ref):
    if dev.leaf != ref["leaf"]:
        # only an exact-arithmetic near-tie may flip the winner
        assert abs(dev.cost - ref["cost"]) <= 1e-13 * abs(ref["cost"]), (dev.leaf, ref["leaf"])
        return
    assert math.isclose(dev.cost, ref["cost"], rel_tol=COST_RTOL)
    assert bool(dev.found) == ref["found"]
    assert max(abs(a - b) for a, b in zip(sum(dev.trajectory(), []), sum(ref["traj"], [])))\
        <= STATE_TOL


@pytest.mark.parametrize("integ", ["qk21", "rect", "qk21+rot", "rect+rot"])
def test_random_problems_vs_oracle(engine, integ):
    """S1 = 8 x 9 = 72 (373,248 leaves) on 6 random problems per mode."""
    rng = np.random.default_rng(5)
    V = np.round(np.arange(0.0, 1.0 + 0.125, 0.125), 3)[:8]
    B = np.round(np.linspace(-1.047, 1.047, 9), 3)
    for _ in range(6):
        st = (float(rng.uniform(-5, 5)), float(rng.uniform(-5, 5)), float(rng.uniform(-3, 3)))
        tg = (float(rng.uniform(-8, 8)), float(rng.uniform(-8, 8)))
        org = (float(rng.uniform(-3, 3)), float(rng.uniform(-3, 3)))
        atan_t = float(np.arctan(tg[0] / tg[1]))
        t_a = float(rng.integers(1, 40)) * 0.05
        ref = O.fulltree_argmin(V, B, st, tg, org, atan_t, 0.5, t_a, t_a + 0.05, 1e18,
                                integ=integ)
        dev = _device_call(engine, V, B, st, tg, org, atan_t, 0.5, t_a, t_a + 0.05, 1e18, integ)
        _agree(dev, ref)
        assert dev.s1 == 72 and dev.found == 1


def test_reference_detail_call(engine, gold):
    """The first recorded reference call (15625 leaves): same winner as the
    reference scan, same cost and states."""
    cfg, det = gold["config"], gold["detail"]
    ep = gold["episodes"][det["episode"]]
    call = ep["calls"][det["call"]]
    t_a = call["pre"]["t"] + cfg["delta_t"]
    costs = np.array(det["leaf_costs"])
    inc = call["pre"]["optimal_criterion"]
    want = int(np.argmin(costs))                 # first index of the minimum
    dev = _device_call(engine, gold["vector_v"], gold["vector_beta"],
                       (call["x"], call["y"], call["phi"]), (ep["x_t"], ep["y_t"]),
                       (ep["x_0"], ep["y_0"]), float(np.arctan(ep["x_t"] / ep["y_t"])),
                       cfg["L"], t_a, t_a + cfg["delta_t"], inc, "qk21")
    assert dev.leaf == want and dev.found == 1
    assert math.isclose(dev.cost, costs[want], rel_tol=COST_RTOL)
    assert max(abs(a - b) for a, b in zip(dev.trajectory()[2],
                                          det["leaf_states_last_layer"][want])) <= STATE_TOL


def test_drop_in_episodes(engine, gold):
    """diplomjourney_amd.run_math_model replays the three reference episodes
    (same seeds, same RNG draws, same stop rule) at the fixtures' grid."""
    from diplomjourney_amd import run_math_model as rmm
    cfg = gold["config"]
    rmm.configure(cfg["delta_v"], cfg["delta_beta"])
    try:
        assert list(rmm.vector_v) == gold["vector_v"]
        assert list(rmm.vector_beta) == gold["vector_beta"]
        for ep in gold["episodes"]:
            recs, stop = rmm.run_episode(ep["seed"], max_calls=6)
            assert (rmm.x_0, rmm.y_0, rmm.phi_0, rmm.x_t, rmm.y_t) == \
                (ep["x_0"], ep["y_0"], ep["phi_0"], ep["x_t"], ep["y_t"])
            assert stop == ep["stop"] and len(recs) == len(ep["calls"])
            assert recs[0]["pre"][5] == ep["first_incumbent"]
            for r, c in zip(recs, ep["calls"]):
                assert r["ret"][3:] == c["ret"][3:]                       # chosen v, beta
                assert max(abs(a - b) for a, b in zip(r["ret"][:3], c["ret"][:3])) <= STATE_TOL
                assert math.isclose(r["optimal_criterion"], c["post"]["optimal_criterion"],
                                    rel_tol=COST_RTOL)
    finally:
        rmm.configure()


@pytest.mark.parametrize("n_shards", [2, 3, 8])
def test_sharded_equals_single_launch(engine, n_shards):
    """Leaf shards (the multi-GPU decomposition) evaluated one after another on
    one GPU + the host selection == one launch, bit for bit."""
    from diplomjourney_amd.abi import MpcFulltreeProblem
    from diplomjourney_amd.distributed import select_fulltree
    from diplomjourney_amd.expansion import fulltree_argmin, fulltree_result
    V = np.round(np.arange(0.0, 1.0 + 0.1, 0.1), 3)
    B = np.round(np.linspace(-1.047, 1.047, 21), 3)
    vg = torch.tensor(V, dtype=torch.float64, device=engine.device)
    bg = torch.tensor(B, dtype=torch.float64, device=engine.device)
    p = MpcFulltreeProblem(0.3, -0.2, 0.5, 4.0, 5.0, 0.0, 0.0, float(np.arctan(0.8)), 0.5,
                           0.1, 0.15)
    one = fulltree_result(fulltree_argmin(engine, p, vg, bg, 1e18, "rect+rot"))
    parts = [fulltree_result(fulltree_argmin(engine, p, vg, bg, 1e18, "rect+rot", s, n_shards))
             for s in range(n_shards)]
    win = select_fulltree(parts, 1e18)
    assert (win.leaf, win.cost, win.found) == (one.leaf, one.cost, one.found)
    assert win.trajectory() == one.trajectory()


def test_batched_episodes_match_reference(engine, gold):
    """The lockstep batched driver (one robot per episode, one batched
    full-tree launch per MPC step) reproduces the three reference episodes."""
    from diplomjourney_amd import run_math_model as rmm
    cfg = gold["config"]
    rmm.configure(cfg["delta_v"], cfg["delta_beta"])
    try:
        starts = [(e["x_0"], e["y_0"], e["phi_0"], e["x_t"], e["y_t"]) for e in gold["episodes"]]
        outs = rmm.run_batched(starts, max_calls=6)
        for (recs, stop), ep in zip(outs, gold["episodes"]):
            assert stop == ep["stop"] and len(recs) == len(ep["calls"])
            assert recs[0]["pre"][5] == ep["first_incumbent"]
            for r, c in zip(recs, ep["calls"]):
                assert r["ret"][3:] == c["ret"][3:]
                assert max(abs(a - b) for a, b in zip(r["ret"][:3], c["ret"][:3])) <= STATE_TOL
                assert math.isclose(r["optimal_criterion"], c["post"]["optimal_criterion"],
                                    rel_tol=COST_RTOL)
    finally:
        rmm.configure()


def test_batched_equals_sequential_episodes(engine):
    """24 random episodes (the script's RNG stream) at S1 = 35: batched
    lockstep driver == one episode after another through predictive_control."""
    from diplomjourney_amd import run_math_model as rmm
    rmm.configure(0.25, math.radians(20))
    try:
        starts = rmm.draw_starts(24, seed=11)
        batched = rmm.run_batched(starts, max_calls=5)
        for s, (recs, stop) in zip(starts, batched):
            rmm.start_episode(*s)
            seq = []
            for _ in range(len(recs)):
                c = rmm.predictive_control(rmm.x, rmm.y, rmm.phi, rmm.v, rmm.x_t, rmm.y_t)
                seq.append((c, rmm.optimal_criterion))
                rmm.x, rmm.y, rmm.phi, rmm.v, rmm.beta = c
            for r, (c, crit) in zip(recs, seq):
                assert r["ret"][3:] == c[3:]
                assert max(abs(a - b) for a, b in zip(r["ret"][:3], c[:3])) <= STATE_TOL
                assert math.isclose(r["optimal_criterion"], crit, rel_tol=COST_RTOL)
    finally:
        rmm.configure()


@pytest.mark.parametrize("integ", ["qk21", "rect+rot"])
def test_device_episodes_equal_lockstep_driver(engine, integ):
    """Workload G's driver, device-resident (run_batched ->
    mpc_fulltree_episodes_run: one block per robot runs its episode's
    full-tree calls back to back in one launch) == the host lockstep driver
    (run_batched_lockstep: one batched full-tree launch per lockstep step, host
    updates), record for record: the same returned states and controls
    (bitwise), incumbents and stops, for 48 of the script's episodes at
    G's grid (S1 = 5 x 13)."""
    from diplomjourney_amd import run_math_model as rmm
    rmm.configure(0.25, math.radians(10))
    try:
        starts = rmm.draw_starts(48, seed=3)
        dev = rmm.run_batched(starts, max_calls=9, integrator=integ)
        ref = rmm.run_batched_lockstep(starts, max_calls=9, integrator=integ)
        assert sum(len(r) for r, _ in dev) > 100
        for (rd, sd), (rr, sr) in zip(dev, ref):
            assert sd == sr and len(rd) == len(rr)
            for a, b in zip(rd, rr):
                assert a["ret"] == b["ret"] and a["optimal_criterion"] == b["optimal_criterion"]
                assert a["pre"] == b["pre"]
        # chunked launches continue the episodes: 4 calls per launch == one launch
        assert rmm.run_batched(starts, max_calls=9, integrator=integ, chunk=4) == dev
    finally:
        rmm.configure()


def test_device_episodes_no_winner_raises_as_the_script(engine, monkeypatch):
    """A first call with no leaf below the first incumbent leaves the script's
    optimal_trajectory at [0] and raises TypeError: both drivers do (the
    first incumbent forced to 0, which no criterion value is below); on the
    device the robot stops after that call with MPC_EP_NO_TRAJ."""
    from diplomjourney_amd import run_math_model as rmm
    from diplomjourney_amd.abi import MPC_EP_NO_TRAJ, MpcFulltreeEpisodeConfig
    from diplomjourney_amd.episode import DeviceFtEpisodes
    rmm.configure(0.25, math.radians(10))
    try:
        starts = rmm.draw_starts(4, seed=5)
        monkeypatch.setattr(rmm._Robot, "_criterion0", lambda self: 0.0)
        for fn in (rmm.run_batched, rmm.run_batched_lockstep):
            with pytest.raises(TypeError):
                fn(starts, max_calls=3, integrator="rect+rot")
        eng, (vg, bg) = rmm._device()
        cfg = MpcFulltreeEpisodeConfig(*starts[0], float(np.arctan(starts[0][3] / starts[0][4])),
                                       0.0, 3, 0)
        ep = DeviceFtEpisodes(eng, [cfg], vg, bg, rmm.L, rmm.delta_t, rmm.eps, "rect+rot")
        ep.run(3)
        calls, stop, _ = ep.read_progress()
        assert calls[0] == 1 and stop[0] & MPC_EP_NO_TRAJ
    finally:
        rmm.configure()


def test_tree_episode_loop_batched_equals_sequential(engine):
    """run_math_model.py's episode loop over the tree expansion (the named
    entry at config.py's resolution, SURVEY Fact 2): R episodes in lockstep
    through the batched kernel (mpc_rollout_argmin_batched) return, call by
    call, exactly what R sequential runs of the drop-in predictive_control
    return (chosen (v, beta) identical, pose within 1e-12), and stop the same
    way."""
    from diplomjourney_amd import math_model_tree as mmt
    from diplomjourney_amd import run_math_model as rmm
    starts = rmm.draw_starts(6, seed=20261015)
    try:
        seq = [rmm.run_tree_episode(s, max_calls=120) for s in starts]
    finally:
        mmt.reset_state()
    bat = rmm.run_tree_batched(starts, max_calls=120, integrator="qk21", engine=engine)
    assert sum(len(r) for r, _ in seq) > 300
    for (rs, ss), (rb, sb) in zip(seq, bat):
        assert ss == sb and len(rs) == len(rb)
        for a, b in zip(rs, rb):
            assert a[3:] == b[3:]
            assert max(abs(p - q) for p, q in zip(a[:3], b[:3])) <= 1e-12


def test_tree_episodes_chunked_launches_equal_one_launch(engine):
    """The device episodes continue across launches: the same episodes run
    7 MPC steps per launch (the log read back after every launch) return
    exactly what one launch per 120 steps returns."""
    from diplomjourney_amd import run_math_model as rmm
    starts = rmm.draw_starts(20, seed=7)
    one = rmm.run_tree_batched(starts, max_calls=120, integrator="qk21", engine=engine)
    many = rmm.run_tree_batched(starts, max_calls=120, integrator="qk21", engine=engine, chunk=7)
    assert one == many
    assert sum(len(r) for r, _ in one) > 200


@pytest.mark.parametrize("integ", ["qk21", "rect+rot"])
def test_batched_episodes_replay_reference_scenario_as_robot_0(engine, scenario, integ):
    """The reference's model run (math_model_tree.py:736: math_mpc from (0, 0,
    0) to (2, 3) with the operator events at p = 60 / 90 / 110, the first
    incumbent of :676) as robot 0 of R = 64 batched device episodes
    (mpc_episodes_run, one block per robot) whose other 63 robots run
    run_math_model.py episodes: robot 0 logs the 151 recorded calls — chosen
    (v, beta) identical, pose within 1e-6, the events and the arrival after
    call 150 — and the other robots equal their sequential drop-in episodes."""
    from diplomjourney_amd import math_model_tree as mmt
    from diplomjourney_amd import run_math_model as rmm
    from diplomjourney_amd.abi import MPC_EP_ARRIVED, MPC_EP_EVENT
    from diplomjourney_amd.episode import (DeviceEpisodes, reference_episode_config,
                                           tree_episode_config)
    calls = [c for c in scenario["calls"] if not c["isActual"]]
    starts = rmm.draw_starts(63, seed=11)
    cfgs = [reference_episode_config(enumerate=True, incumbent0=10000050990.195135)]
    cfgs += [tree_episode_config(s, 60) for s in starts]
    eps = DeviceEpisodes(engine, cfgs, 3, integ, log_capacity=256)
    eps.run(400)
    n, stop, _ = eps.read_progress()
    logs = eps.read_logs()
    assert n[0] == len(calls) == 151 and stop[0] & MPC_EP_ARRIVED
    worst = 0.0
    for i, (rec, g) in enumerate(zip(calls, logs[0])):
        assert (g["p"], g["episode"], g["found"]) == (i + 1, 1, int(rec["found"])), i
        assert (g["v"], g["beta"]) == tuple(rec["ret"][3:5]), i
        worst = max(worst, max(abs(a - b) for a, b in zip((g["x"], g["y"], g["phi"]),
                                                          rec["ret"][:3])))
        want = MPC_EP_EVENT if g["p"] in (60, 90, 110) else 0
        want |= MPC_EP_ARRIVED if i == len(calls) - 1 else 0
        assert g["status"] == want, (i, g["status"])
    assert worst <= 1e-6, worst
    if integ == "qk21":
        try:
            for r in (1, 2, 3, 40):
                seq, st = rmm.run_tree_episode(starts[r - 1], max_calls=60)
                got = logs[r]
                assert len(seq) == len(got) == n[r]
                for a, g in zip(seq, got):
                    assert a[3:] == [g["v"], g["beta"]]
                    assert max(abs(p - q) for p, q in zip(a[:3], (g["x"], g["y"], g["phi"]))) <= 1e-12
        finally:
            mmt.reset_state()
