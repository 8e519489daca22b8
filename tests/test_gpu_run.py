"""GPU: the persistent run (mpc_episode_run, csrc/mpc_run.h) — K complete MPC
steps of the one-GPU chained episode in one launch — logs, state and winner
record bit for bit equal to the same steps as chained launches + their flush
(which tests/test_gpu_parity.py pins to the two-launch episode and, at config
C's size, to the qk21 oracle).  The reference loop is math_mpc
(math_model_tree.py:515-635) over predictive_control (:278-496)."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu


def _pool(engine, n, ns, count, seed, tiled=False):
    from diplomjourney_amd import math_model_tree as mmt
    V = torch.tensor(mmt.vector_of_velocities(0.5), dtype=torch.float64, device="cuda")
    B = torch.tensor(mmt.vector_of_beta_angles(0.0), dtype=torch.float64, device="cuda")
    if tiled:
        return [engine.sample_controls_tiled(V, B, n, ns, seed + i) for i in range(count)]
    return [engine.sample_controls(V, B, n, ns, seed + i) for i in range(count)]


def _log(ep):
    return [(r.step, r.index, r.cost, r.x, r.y, r.phi, r.v, r.beta, r.p, r.episode, r.status)
            for r in ep.read_log()]


def _episode(engine, n, ns, wheelbase=None, max_steps=None, cap=512):
    from diplomjourney_amd.episode import DeviceEpisode
    ep = DeviceEpisode(engine, n, ns, integrator="rect+cum", log_capacity=cap, chain=True,
                       L=wheelbase)
    if max_steps:
        ep.cfg.max_steps = max_steps
        ep.reset()
    return ep


def _chained(engine, n, ns, batches, **kw):
    ep = _episode(engine, n, ns, **kw)
    for c in batches:
        ep.step(controls=c)
    ep.flush()
    return ep


def _state_bytes(ep):
    torch.cuda.synchronize()
    return bytes(ep.state.cpu().numpy().tobytes()), bytes(ep.local.cpu().numpy().tobytes())


@pytest.mark.parametrize("wheelbase,n,ns", [(0.5, 50_000, 10), (0.45, 50_000, 10),
                                            (0.5, 100_000, 3), (0.45, 60_000, 3)])
def test_run_matches_chained_steps(engine, wheelbase, n, ns):
    """130 steps with the operator events (p = 60 / 90 / 110) as ONE run call
    (three launches: 64 + 64 + 2 steps) equal 130 chained steps + flush: the
    log records, the episode state and the last winner's result record; a
    partial last tile (50_000 = 97 x 512 + 336); both wheelbase forms."""
    steps = 130
    pool = _pool(engine, n, ns, 8, 500)
    batches = [pool[i % 8] for i in range(steps)]
    ch = _chained(engine, n, ns, batches, wheelbase=wheelbase)
    want = _log(ch)
    assert len(want) == steps and {r[8] for r in want} >= {60, 90, 110}
    ru = _episode(engine, n, ns, wheelbase=wheelbase)
    ru.run(batches)
    assert _log(ru) == want
    assert ru.chain_error() == 0
    st_ch, out_ch = _state_bytes(ch)
    st_ru, out_ru = _state_bytes(ru)
    assert out_ru == out_ch
    # the head, the stale trajectory and the early-publication inputs (the
    # chain bookkeeping after them — tags, counters — differs by design)
    from diplomjourney_amd import native
    head = 8 * 64
    assert st_ru[:head] == st_ch[:head]
    assert native.lib() is not None


@pytest.mark.parametrize("ns", [2, 3, 12])
def test_run_restart_and_horizons(engine, ns):
    """Episode restarts (step limit 40) inside a run — the tiles' speculated
    step size is then wrong and their loop reruns with the published one —
    and the horizons around the head prefetch (N = 2, 3) and config D's N =
    12: 60 steps, runs of 7 + 53, equal the chained steps."""
    n, steps = 20_000, 60
    pool = _pool(engine, n, ns, 4, 900 + ns)
    batches = [pool[i % 4] for i in range(steps)]
    want = _log(_chained(engine, n, ns, batches, max_steps=40))
    assert len({r[9] for r in want}) >= 2, "no episode restart exercised"
    ru = _episode(engine, n, ns, max_steps=40)
    ru.run(batches[:7])
    ru.run(batches[7:])
    assert _log(ru) == want
    assert ru.chain_error() == 0


def test_run_tiled_config_c_graph_replay(engine):
    """Config C's shape (1e6 x N = 10, tiled controls, 1954 units per step):
    a run captured in a HIP graph and replayed twice (the replay repeats the
    run's epochs: the tags, the records and the claim counter must be back to
    zero between launches) equals 2 x 12 chained steps + flush on the same
    batches, mixed with chained steps before it."""
    n, ns, k = 1_000_000, 10, 12
    pool = _pool(engine, n, ns, 4, 77, tiled=True)
    batches = [pool[i % 4] for i in range(k)]
    ch = _chained(engine, n, ns, batches[:3] + batches + batches)
    want = _log(ch)
    ru = _episode(engine, n, ns)
    for c in batches[:3]:
        ru.step(controls=c)               # chained steps first; run() flushes them
    ru.flush()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    n0 = ru.steps_enqueued
    with torch.cuda.graph(g):
        ru.run(batches)
    ru.steps_enqueued = n0
    g.replay()
    g.replay()
    ru.steps_enqueued += 2 * k
    assert _log(ru) == want
    assert ru.chain_error() == 0
    ws = ru._run_ws.cpu()
    assert int(ws.count_nonzero()) == 0, "the run left its workspace dirty"


def test_run_many_units_per_step(engine):
    """1.1e6 candidates = 2149 units per step (> 2048: the selector polls its
    records in two chunks) equal the chained steps."""
    n, ns, steps = 1_100_000, 6, 5
    pool = _pool(engine, n, ns, steps, 700)
    want = _log(_chained(engine, n, ns, pool, cap=16))
    ru = _episode(engine, n, ns, cap=16)
    ru.run(pool)
    assert _log(ru) == want
    assert ru.chain_error() == 0


def test_run_wheelbase_mismatch_and_arguments(engine):
    """A cfg whose wheelbase form differs from the state's sets chain error 2;
    the entry's argument checks (epoch 0, misaligned controls, too small a
    workspace) refuse without launching."""
    from diplomjourney_amd import abi, native
    n, ns = 20_000, 10
    pool = _pool(engine, n, ns, 2, 40)
    ep = _episode(engine, n, ns, cap=16)
    ep.run(pool)
    assert ep.chain_error() == 0
    L = native.lib()
    v, b = pool[0]
    V = (ctypes.c_void_p * 1)(v.data_ptr())
    B = (ctypes.c_void_p * 1)(b.data_ptr())
    Bm = (ctypes.c_void_p * 1)(b.data_ptr() + 8)

    def call(e0=1, bp=B, wsb=None, integ=None):
        return L.mpc_episode_run(ctypes.byref(ep.cfg), ep.state.data_ptr(), e0, V, bp, 1, n, ns, 0,
                                 ep._integ if integ is None else integ, ep._run_ws.data_ptr(),
                                 ep._run_ws.numel() if wsb is None else wsb,
                                 ep.local.data_ptr(), ep.log.data_ptr(), 16, None)

    assert call(e0=0) == abi.MPC_ERR_ARG
    assert call(bp=Bm) == abi.MPC_ERR_UNSUPPORTED
    assert call(wsb=ep._run_ws.numel() - 1) == abi.MPC_ERR_WORKSPACE
    assert call(integ=abi.INTEGRATORS["rect"]) == abi.MPC_ERR_UNSUPPORTED
    torch.cuda.synchronize()
    ep.cfg.L = 0.45                      # state reset with L = 0.5
    ep.run(pool[1:])
    assert ep.chain_error() == 2
