"""Parity legs of bench.py: the run's own hot-path forms re-checked against the
CPU oracle after every timed region.

TEST INFRASTRUCTURE ONLY (the checker).  Imported by bench.py's parity pass
and tests/ — never by the product package, never inside a timed region.
Everything compared here comes from the product's C-ABI on the GPU; the
expected values come from oracle/mpc_oracle.c in qk21 mode (scipy quad's
21-point Kronrod sums, glibc trig, the reference's operation order — pinned
bitwise to the reference's own outputs by tests/test_oracle_golden.py) and
from the host restatement of the episode bookkeeping below.

Legs:
  episode_leg        a15-a17 + f1: a device-resident math_mpc episode of the
                     bench's own step form, against an INDEPENDENT oracle
                     episode: the oracle scans every step's batch itself, on
                     the problem built from ITS OWN previous winner (not the
                     device's log), runs the finishing logic, the operator
                     events and the restart itself — so chosen index, (v, beta),
                     the returned pose and the status bits are all compared,
                     and pose drift would show.
  sampler_leg        f2: the bench's resident batch (tiled sampler) and the
                     device sampler's per-step batches of a sampled-mode
                     episode, bitwise against the oracle sampler on the grid
                     the oracle episode rebuilds (math_model_tree.py:239-256,
                     slow-down :312-316), and each sampled step's winner.
  fulltree_leg       f3: one S1 = 451 full-tree MPC step
                     (run_math_model.py:156-197) against the oracle's scan,
                     split over threads and ranks by first-layer control.
  ft_episodes_leg    f4: run_math_model.py's episode loop (:231-280), device
                     resident (mpc_fulltree_episodes_run), against the oracle
                     driving the same episodes call by call.
  tree_episodes_leg  the named entry over the tree expansion
                     (mpc_episodes_run, workload R) against the oracle driving
                     the same episodes with math_model_tree.py's step.
"""
import math
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from oracle import oracle as O

INC_MAX = float(sys.maxsize)          # optimal_criterion = sys.maxsize (:428)
# status bits of mpc_episode_log_t (include/mpc_rollout.h)
STALE, STUCK, BREAK, EVENT, ARRIVED, LIMIT = 1, 2, 4, 8, 16, 32
ROW = 13                              # cost, index, v, beta, 3 layer states x 3


class ShardScanner:
    """One rank's candidates of one batch as host SoA, pre-split into
    contiguous column chunks (one per thread); scan() is the oracle's
    strict-< first minimum over the shard (mpc_oracle_rollout_argmin per
    chunk, lexicographic (cost, index) over the chunks: the sequential scan's
    winner)."""

    def __init__(self, v, b, index_base, threads):
        n = v.shape[1]
        cuts = np.linspace(0, n, max(1, min(threads, n)) + 1).astype(np.int64)
        self.chunks = [(int(index_base + a), np.ascontiguousarray(v[:, a:z]),
                        np.ascontiguousarray(b[:, a:z])) for a, z in zip(cuts[:-1], cuts[1:])
                       if z > a]
        self.n_steps = v.shape[0]

    def scan(self, ex, prob, integ="qk21"):
        """Row [cost, index, v, beta, layers 0..2 (x, y, phi)] of the shard's
        first minimum (cost = inf, index = -1 when nothing is finite)."""
        futs = [ex.submit(O.rollout_argmin, prob, v, b, index_base=base, integ=integ)
                for base, v, b in self.chunks]
        best = None
        for f in futs:
            r = f.result()[0]
            if r.index >= 0 and (best is None or (r.cost, r.index) < (best.cost, best.index)):
                best = r
        row = np.full(ROW, np.nan)
        if best is None:
            row[0], row[1] = math.inf, -1
            return row
        last = self.n_steps - 1
        row[:4] = best.cost, best.index, best.v, best.beta
        for k in range(3):
            row[4 + 3 * k:7 + 3 * k] = best.traj[min(k, last)][:3]
        return row


def global_winner(rows):
    """rows [world, ROW]: the lexicographic (cost, index) minimum over the
    ranks' rows (contiguous shards: the single-device scan's first minimum)."""
    ok = [r for r in rows if r[1] >= 0]
    if not ok:
        return rows[0]
    return min(ok, key=lambda r: (r[0], r[1]))


class OracleMpcEpisode:
    """math_mpc's loop (math_model_tree.py:515-635) restated on the host for
    the checker, with the device episode's constants (mpc_episode_config_t):
    the start of an episode (:521-541, first incumbent :676), per step
    t += delta_t (:302), the winner taken into optimal_trajectory /
    result_v / result_beta only when it beats the incumbent (:351-359, stale
    otherwise), the finishing logic m (:392-414), the incumbent reset to
    sys.maxsize (:428), the stuck detector (:559-563), the operator events at
    cfg.p_turn_right / p_turn_left / p_new_target (:564-569 with :118-226),
    p += 1, the loop condition (:542) and the step limit; an ended episode
    restarts (the bench's episode stream).  Event targets use the drop-in's
    _turn_target (math_model_tree.py:181-204, pinned by the reference
    scenario's event calls in the CPU suite)."""

    def __init__(self, cfg):
        self.c = cfg
        self.episodes = 0
        self.has_traj = False
        self.ot = [[0.0] * 3 for _ in range(3)]
        self.ot_v = self.ot_beta = 0.0
        self.restart()

    def restart(self):
        c = self.c
        self.x, self.y, self.phi = c.start_x, c.start_y, c.start_phi
        self.v, self.beta = c.start_v, c.start_beta
        self.xt, self.yt = c.target_x, c.target_y
        self.x0, self.y0 = c.start_x, c.start_y
        self.t, self.p, self.m, self.slowing = 0.0, 1, 0, 0
        self.episodes += 1
        self.recursive = False
        self.incumbent = (c.incumbent0 if c.incumbent0 != 0.0 else
                          O.cost(self.x0, self.y0, self.xt, self.yt, self.x0, self.y0))

    def begin_step(self):
        """(mpc_problem_t, incumbent) of the next step (t advanced)."""
        from diplomjourney_amd.abi import make_problem
        self.t = self.t + self.c.delta_t
        return (make_problem(self.x, self.y, self.phi, self.xt, self.yt, self.x0, self.y0,
                             self.c.L, self.t, self.t + self.c.delta_t), self.incumbent)

    def grids(self):
        """The step's (V, B) (:239-256) around the current control with the
        slow-down override (:312-316), and its sampler seed."""
        from diplomjourney_amd import math_model_tree as mmt
        V = mmt.vector_of_velocities(self.v)
        B = mmt.vector_of_beta_angles(self.beta)
        if self.slowing > 0 and V:
            vel = min(V) if min(V) > self.c.v_min else self.c.v_min
            V = [vel] * len(V)
        seed = (self.c.seed + 0x9E3779B9 * (self.p + 1000 * self.episodes)) & (2 ** 64 - 1)
        return V, B, seed

    def advance(self, row, incumbent):
        """Apply the step's global winner row; returns the expected log
        record (index, found, p, episode, status, x, y, phi, v, beta, cost)."""
        from diplomjourney_amd import math_model_tree as mmt
        c = self.c
        found = row[1] >= 0 and row[0] < incumbent
        rec = {"index": int(row[1]) if found else -1, "found": int(found), "p": self.p,
               "episode": self.episodes, "cost": float(row[0])}
        self.slowing -= 1
        self.incumbent = INC_MAX
        status = 0
        if found:
            self.ot = [list(row[4 + 3 * k:7 + 3 * k]) for k in range(3)]
            self.ot_v, self.ot_beta = float(row[2]), float(row[3])
            self.has_traj = True
        else:
            status |= STALE
            if not self.has_traj:        # [[[0]]]: no layer states, stay at the pose
                self.ot = [[self.x, self.y, self.phi] for _ in range(3)]
                self.ot_v, self.ot_beta = self.v, self.beta
        k = 0
        if self.m == 2:
            k = 2
        elif self.m == 1:
            k = 1
            self.m += 1
        elif mmt.is_on_target(self.ot[2][0], self.ot[2][1], self.xt, self.yt)[0]:
            self.m += 1
        x_prev, y_prev = self.x, self.y
        self.x, self.y, self.phi = self.ot[k]
        self.v, self.beta = self.ot_v, self.ot_beta
        ended = False
        if self.recursive:                               # :559-561
            status |= BREAK
            ended = True
        else:
            if self.x == x_prev and self.y == y_prev:    # :562-563
                self.recursive = True
                status |= STUCK
            for p_ev, sign in ((c.p_turn_right, -1), (c.p_turn_left, +1)):
                if self.p == p_ev:
                    self.xt, self.yt = mmt._turn_target(self.x, self.y, self.phi,
                                                        c.turn_distance, sign)
                    self.x0, self.y0 = self.x, self.y
                    self.slowing = c.slow_turn
                    status |= EVENT
            if self.p == c.p_new_target:
                self.xt, self.yt = c.event_target_x, c.event_target_y
                self.x0, self.y0 = self.x, self.y
                self.slowing = c.slow_new_target
                status |= EVENT
            self.p += 1
            if mmt.is_on_target(self.x, self.y, self.xt, self.yt)[0]:     # :542
                status |= ARRIVED
                ended = True
            elif c.max_steps > 0 and self.p > c.max_steps:
                status |= LIMIT
                ended = True
        rec.update(status=status, x=self.x, y=self.y, phi=self.phi, v=self.v, beta=self.beta)
        if ended:
            self.restart()
        return rec


def compare_records(logged, want, rows_oracle):
    """Per-step comparison of device log records with the oracle episode's."""
    same = vb = status = pe = 0
    pose = cost = 0.0
    first_bad = None
    for i, (r, w) in enumerate(zip(logged, want)):
        ok = r.index == w["index"] and r.found == w["found"]
        same += ok
        if ok and (r.v, r.beta) == (w["v"], w["beta"]):
            vb += 1
        status += r.status == w["status"]
        pe += (r.p, r.episode) == (w["p"], w["episode"])
        pose = max(pose, abs(r.x - w["x"]), abs(r.y - w["y"]), abs(r.phi - w["phi"]))
        if ok and r.found and math.isfinite(w["cost"]):
            cost = max(cost, abs(r.cost - w["cost"]) / abs(w["cost"]))
        if not ok and first_bad is None:
            first_bad = {"step": i, "device_index": int(r.index), "oracle_index": w["index"],
                         "oracle_cost": w["cost"]}
    n = max(1, len(want))
    return {"identity_rate": same / n, "v_beta_identical_rate": vb / n,
            "status_identical_rate": status / n, "p_episode_identical_rate": pe / n,
            "max_abs_pose_diff": pose, "max_rel_cost_diff": cost, "first_mismatch": first_bad}


def episode_leg(fresh_episode, batches, scanners, allgather, threads):
    """The device episode `fresh_episode` (already stepped over `batches` and
    its log read: fresh_episode[1]) against OracleMpcEpisode on the same
    controls: scanners[i % len(scanners)] holds batch i's shard on this rank.
    allgather(np.ndarray) -> [world, ...] (identity on one rank)."""
    cfg, log = fresh_episode
    oe = OracleMpcEpisode(cfg)
    want = []
    t0 = time.perf_counter()
    with ThreadPoolExecutor(max_workers=threads) as ex:
        for i in range(len(log)):
            prob, inc = oe.begin_step()
            row = scanners[i % len(scanners)].scan(ex, prob)
            want.append(oe.advance(global_winner(allgather(row)), inc))
    out = compare_records(log, want, None)
    out.update(steps=len(log),
               event_steps=sum(1 for w in want if w["status"] & EVENT),
               events_at_p=sorted({w["p"] for w in want if w["status"] & EVENT}),
               restarts=sum(1 for w in want if w["status"] & (ARRIVED | LIMIT | BREAK)),
               stale_steps=sum(1 for w in want if w["status"] & STALE),
               check_s=time.perf_counter() - t0)
    return out


def sampled_leg(cfg, batches_dev, logged, n_local, n_steps, lo, allgather, threads):
    """Sampled-mode steps: batches_dev[i] = this rank's (v, beta) host arrays
    the device sampler drew for step i; logged = the device log.  Each batch
    must equal the oracle sampler's on the grid and seed the oracle episode
    rebuilds (bitwise), and each step's winner the oracle's."""
    oe = OracleMpcEpisode(cfg)
    want, bitwise = [], []
    with ThreadPoolExecutor(max_workers=threads) as ex:
        for v_dev, b_dev in batches_dev:
            V, B, seed = oe.grids()
            ov, ob = O.sample_controls(V, B, n_local, n_steps, seed, index_base=lo)
            bitwise.append(bool(np.array_equal(ov, v_dev) and np.array_equal(ob, b_dev)))
            prob, inc = oe.begin_step()
            row = ShardScanner(ov, ob, lo, threads).scan(ex, prob)
            want.append(oe.advance(global_winner(allgather(row)), inc))
    all_bitwise = bool(np.all(allgather(np.array(bitwise, dtype=np.float64)) == 1.0))
    out = compare_records(logged, want, None)
    out.update(steps=len(batches_dev), batches_bitwise=all_bitwise)
    return out


def fulltree_leg(dev_results, V, B, problem, incumbent, rank, world, allgather, threads):
    """One full-tree MPC step: the device's results {integrator: (leaf, cost,
    found, traj)} against the oracle's qk21 scan, split by first-layer control
    over ranks (contiguous k0 ranges) and threads."""
    t0 = time.perf_counter()
    s1 = len(V) * len(B)
    lo, hi = rank * s1 // world, (rank + 1) * s1 // world
    cuts = np.linspace(lo, hi, max(1, min(threads, hi - lo)) + 1).astype(np.int64)
    st, tg, org, atan_t, L, t_a, t_b = problem
    with ThreadPoolExecutor(max_workers=threads) as ex:
        futs = [ex.submit(O.fulltree_argmin_range, V, B, int(a), int(z), st, tg, org, atan_t, L,
                          t_a, t_b) for a, z in zip(cuts[:-1], cuts[1:]) if z > a]
        parts = [f.result() for f in futs]
    row = np.full(11, np.nan)
    row[0], row[1] = math.inf, -1
    for leaf, cost, traj in parts:
        if leaf >= 0 and (cost, leaf) < (row[0], row[1]):
            row[0], row[1] = cost, leaf
            row[2:] = np.array(traj).ravel()
    best = global_winner(allgather(row))
    found = best[1] >= 0 and best[0] < incumbent
    out = {"s1": s1, "leaves": s1 ** 3, "oracle_leaf": int(best[1]), "oracle_found": bool(found),
           "check_s": None}
    for integ, (leaf, cost, dfound, traj) in dev_results.items():
        d = max(abs(a - b) for a, b in zip(np.array(traj).ravel(), best[2:]))
        out[integ] = {"leaf_identical": int(leaf) == int(best[1]),
                      "found_identical": bool(dfound) == bool(found),
                      "rel_cost_diff": abs(cost - best[0]) / abs(best[0]),
                      "max_abs_state_diff": float(d)}
    out["check_s"] = time.perf_counter() - t0
    return out


def _ft_criterion0(x0, y0, phi0, xt, yt):
    """control_criterion([x_0, y_0, phi_0]) of run_math_model.py:82-86 at the
    episode's start (the line origin: distance_from_line = 1000, :53-55)."""
    return O.fulltree_cost(x0, y0, phi0, xt, yt, x0, y0, float(np.arctan(xt / yt)))


def ft_episodes_oracle(starts, V, B, L, delta_t, eps, max_calls, threads):
    """run_math_model.py's loop (:231-280) per start on the oracle: per call
    t += delta_t (:156), the S1^3 scan against the never-reset incumbent
    (:193-196), optimal_trajectory[0][0] of the last winner returned (stale
    when none wins), the on-target test (:241) and the two-non-move stop
    (:266-272).  Returns [(records [x, y, phi, v, beta, criterion], stop)]."""
    nb = len(B)
    s1 = len(V) * nb

    def one(s):
        x0, y0, phi0, xt, yt = s
        atan_t = float(np.arctan(xt / yt))
        crit = _ft_criterion0(x0, y0, phi0, xt, yt)
        x, y, phi, t, k = x0, y0, phi0, 0.0, 0
        prev, stale, recs = (x, y), None, []
        while not (xt - x) ** 2 + (yt - y) ** 2 <= eps:
            if len(recs) == max_calls:
                return recs, "max_calls"
            t = t + delta_t
            r = O.fulltree_argmin(V, B, (x, y, phi), (xt, yt), (x0, y0), atan_t, L, t,
                                  t + delta_t, crit)
            if r["found"]:
                crit = r["cost"]
                k0 = r["leaf"] // (s1 * s1)
                stale = r["traj"][0] + [float(V[k0 // nb]), float(B[k0 % nb])]
            if stale is None:
                return recs, "no_traj"
            recs.append(list(stale) + [crit])
            x, y, phi = stale[:3]
            if (x, y) == prev:
                k += 1
            if k == 2:
                return recs, "recursive_error"
            prev = (x, y)
        return recs, "on_target"

    with ThreadPoolExecutor(max_workers=threads) as ex:
        return list(ex.map(one, starts))


def compare_episodes(dev, ref):
    """[(records, stop)] of the device against the oracle's: stops, call
    counts and (v, beta) identical; poses and criteria."""
    calls = same_ctl = 0
    stops = all(sd == sr for (_, sd), (_, sr) in zip(dev, ref))
    lens = all(len(rd) == len(rr) for (rd, _), (rr, _) in zip(dev, ref))
    pose = crit = 0.0
    for (rd, _), (rr, _) in zip(dev, ref):
        for a, b in zip(rd, rr):
            calls += 1
            same_ctl += a[3:5] == b[3:5]
            pose = max(pose, max(abs(p - q) for p, q in zip(a[:3], b[:3])))
            if len(a) > 5 and len(b) > 5:
                crit = max(crit, abs(a[5] - b[5]) / abs(b[5]))
    return {"episodes": len(ref), "calls": calls, "stops_identical": stops,
            "calls_identical": lens, "v_beta_identical_rate": same_ctl / max(1, calls),
            "max_abs_pose_diff": pose, "max_rel_criterion_diff": crit}


def tree_episodes_oracle(starts, max_calls, threads):
    """run_math_model.py's loop (:231-280) over math_model_tree.py's MPC step
    (the named entry at the reference's resolution, SURVEY Fact 2) per start
    on the oracle: the grid around the current (v, beta) (:239-256), the
    |V| x |B| constant sequences k = a*|B| + b (:308-360), N = 3, qk21, the
    first incumbent of the start's line origin (:252), sys.maxsize after every
    call (:428), the finishing logic m (:392-414), the on-target test and the
    two-non-move stop (:266-272).  Returns [(records [x, y, phi, v, beta],
    stop)]."""
    from diplomjourney_amd import math_model_tree as mmt
    from diplomjourney_amd.abi import make_problem

    def one(s):
        x0, y0, phi0, xt, yt = s
        x, y, phi, v, b = x0, y0, phi0, 0.0, 0.0
        inc = O.cost(x0, y0, xt, yt, x0, y0)
        t, m, k, prev, recs = 0.0, 0, 0, (x, y), []
        ot = None
        while not (xt - x) ** 2 + (yt - y) ** 2 <= mmt.eps:
            if len(recs) == max_calls:
                return recs, "max_calls"
            V, Bg = mmt.vector_of_velocities(v), mmt.vector_of_beta_angles(b)
            vs = np.tile(np.repeat(np.array(V, dtype=np.float64), len(Bg)), (3, 1))
            bs = np.tile(np.tile(np.array(Bg, dtype=np.float64), len(V)), (3, 1))
            t = t + mmt.delta_t
            r = O.rollout_argmin(make_problem(x, y, phi, xt, yt, x0, y0, mmt.L, t,
                                              t + mmt.delta_t), vs, bs, incumbent=inc)[0]
            inc = INC_MAX
            if r.found:
                ot = [list(r.traj[q][:3]) for q in range(3)] + [[r.v, r.beta]]
            if ot is None:
                return recs, "no_traj"
            q = 0
            if m == 2:
                q = 2
            elif m == 1:
                q, m = 1, 2
            elif (xt - ot[2][0]) ** 2 + (yt - ot[2][1]) ** 2 <= mmt.eps:
                m += 1
            x, y, phi = ot[q]
            v, b = ot[3]
            recs.append([x, y, phi, v, b])
            if (x, y) == prev:
                k += 1
            if k == 2:
                return recs, "recursive_error"
            prev = (x, y)
        return recs, "on_target"

    with ThreadPoolExecutor(max_workers=threads) as ex:
        return list(ex.map(one, starts))
