"""Drop-in for run_math_model.py's full-tree MPC on MI355X.

Same module surface as the reference script's definitions
(run_math_model.py:1-229): the grids `vector_v` / `vector_beta` (:24-33), the
module globals read by the criterion (`x_0, y_0, x_t, y_t, t`,
`optimal_criterion`, `optimal_trajectory`), `is_on_target`,
`get_distance_from_line`, `get_distance_from_target`, `saturation`,
`control_criterion` and `predictive_control(_initial_x, _initial_y,
_initial_phi, _initial_velocity, _target_x, _target_y)` with the same return
value.  `predictive_control` evaluates all S1^3 leaves of the tree in ONE
C-ABI call (`mpc_fulltree_argmin`, include/mpc_rollout.h) instead of the
three Python layer loops (:158-197), keeping the reference's incumbent rule:
`optimal_criterion` is NOT reset between calls of an episode (:193-196), and
when no leaf beats it the previous winner's first-layer state is returned
again (the reference re-reads its stale `optimal_trajectory`).

`run_episode` re-enacts one iteration of the script's episode loop
(:231-280) without the plotting; `configure(delta_v, delta_beta)` rebuilds
the grids for a different control resolution (at the reference's config the
tree has S1^3 = 1.4e13 leaves, SURVEY Fact 2).
"""
import math

import numpy as np
import torch

from . import config as _cfg
from .abi import MpcFulltreeProblem
from .expansion import (Expansion, fulltree_argmin, fulltree_argmin_batched, fulltree_result,
                        fulltree_results)

L = _cfg.L
delta_t = _cfg.delta_t
beta_max = _cfg.beta_max
v_max = _cfg.v_max
eps = _cfg.eps

# Actual (:13-19)
beta = 0
v = 0
phi = _cfg.phi_0
x = _cfg.x_0
y = _cfg.y_0
x_0, y_0, phi_0 = _cfg.x_0, _cfg.y_0, _cfg.phi_0
x_t, y_t = _cfg.x_t, _cfg.y_t

prediction_horizon = 3
INTEGRATOR = "qk21"        # the reference's quad() arithmetic; "rect", "+rot" as in the ABI

vector_v = vector_beta = None
size_max_1 = size_max_2 = size_max_3 = 0
t = 0
optimal_trajectory = [0]
optimal_criterion = None

_engine = None
_grids_dev = None
_group = None            # torch.distributed group when the leaves are sharded over ranks


def shard_over(group=None):
    """Shard every predictive_control's leaves over the ranks of `group`
    (torch.distributed, one process per GPU): each rank evaluates a contiguous
    leaf range, one all_gather of the 200-B results selects the winner on
    every rank.  shard_over(None) returns to single-device evaluation."""
    global _group
    _group = group


def configure(delta_v=_cfg.delta_v, delta_beta=_cfg.delta_beta):
    """The grids of :24-33 for a control resolution (defaults: config.py)."""
    global vector_v, vector_beta, size_max_1, size_max_2, size_max_3, _grids_dev
    vector_v = np.round(np.arange(0, v_max + delta_v, delta_v), 3)   # v = 0 at import (:14)
    vector_beta = np.round(np.arange(-beta_max, beta_max + delta_beta, delta_beta), 3)
    size_max_1 = np.size(vector_beta) * np.size(vector_v)
    size_max_2 = pow(size_max_1, 2)
    size_max_3 = pow(size_max_1, 3)
    _grids_dev = None


configure()


def is_on_target(actual_x, actual_y, target_x, target_y):
    return (target_x - actual_x) ** 2 + (target_y - actual_y) ** 2 <= eps


def get_distance_from_line(x_a, y_a):
    if x_a == x_0 and y_a == y_0:
        return 1000
    return (abs((y_t - y_0) * x_a - (x_t - x_0) * y_a + x_t * y_0 - y_t * x_0)
            / (math.sqrt((y_t - y_0) ** 2 + (x_t - x_0) ** 2)))


def get_distance_from_target(x_a, y_a):
    return math.sqrt((x_t - x_a) ** 2 + (y_t - y_a) ** 2)


def saturation(value, value_mplt):
    if value > value_mplt:
        value = value_mplt
    elif value < -value_mplt:
        value = -value_mplt
    return value


def control_criterion(predicted_coordinates):
    """:82-86, host scalar (the episode's first incumbent); the leaves are
    scored on the device by the same expression (csrc/mpc_fulltree.h)."""
    angle_from_line = (np.arctan(x_t / y_t) - predicted_coordinates[2])
    distance_from_target = get_distance_from_target(predicted_coordinates[0],
                                                    predicted_coordinates[1])
    distance_from_line = get_distance_from_line(predicted_coordinates[0],
                                                predicted_coordinates[1])
    return 10000 * distance_from_target + 10 * angle_from_line ** 2 + 100 * distance_from_line ** 2


def _device():
    global _engine, _grids_dev
    if _engine is None:
        _engine = Expansion("cuda")
    if _grids_dev is None:
        _grids_dev = (torch.tensor(np.asarray(vector_v, dtype=np.float64), device=_engine.device),
                      torch.tensor(np.asarray(vector_beta, dtype=np.float64),
                                   device=_engine.device))
    return _engine, _grids_dev


def predictive_control(_initial_x, _initial_y, _initial_phi, _initial_velocity, _target_x,
                       _target_y):
    """:133-228 — one MPC step over the full tree; returns [x, y, phi, v, beta]
    of the best leaf's first layer.  (_initial_velocity, _target_* are unused
    by the reference's expansion as well.)"""
    global optimal_trajectory, optimal_criterion, t
    t += delta_t                                                   # :156
    eng, (vg, bg) = _device()
    p = MpcFulltreeProblem(float(_initial_x), float(_initial_y), float(_initial_phi),
                           float(x_t), float(y_t), float(x_0), float(y_0),
                           float(np.arctan(x_t / y_t)), float(L), float(t),
                           float(t + delta_t))
    if _group is None:
        r = fulltree_result(fulltree_argmin(eng, p, vg, bg, optimal_criterion, INTEGRATOR))
    else:
        import torch.distributed as dist
        from .distributed import gather_bytes, select_fulltree
        rank, world = dist.get_rank(_group), dist.get_world_size(_group)
        local = fulltree_argmin(eng, p, vg, bg, optimal_criterion, INTEGRATOR, rank, world)
        gathered = gather_bytes(local, _group)
        r = select_fulltree(gathered.cpu().numpy().tobytes(), optimal_criterion)
    if r.found:
        optimal_criterion = r.cost
        optimal_trajectory = [[r.trajectory()[i] + ([r.v[0], r.beta[0]] if i == 0 else [])
                               for i in range(3)]]
    # the reference reads optimal_trajectory[0][0] whether or not it changed
    # (an int 0 before any winner: the same TypeError as the script)
    first = optimal_trajectory[0][0]
    return [first[0], first[1], first[2], first[3], first[4]]


def start_episode(x0, y0, phi0, xt, yt):
    """The per-episode resets of :232-246 (plotting omitted)."""
    global t, v, x_0, y_0, phi_0, x_t, y_t, x, y, phi, optimal_trajectory, optimal_criterion
    t = 0
    v = 0
    x_0, y_0, phi_0, x_t, y_t = x0, y0, phi0, xt, yt
    x, y, phi = x_0, y_0, phi_0
    optimal_trajectory = [0]
    optimal_criterion = control_criterion([x_0, y_0, phi_0])


def run_episode(seed=None, max_calls=None):
    """One iteration of the :231-280 episode loop: random start and target
    from numpy's global RNG (seeded here when `seed` is given), MPC steps until
    on target, two non-moves ("Recursive error", :267-270) or `max_calls`.
    Returns (records, stop) with one (x, y, phi, v) -> result record per step."""
    global x, y, phi, v, beta
    if seed is not None:
        np.random.seed(seed)
    x0 = np.random.uniform(-10, 10)
    y0 = np.random.uniform(-10, 10)
    phi0 = np.random.uniform(-math.pi, math.pi)
    xt = np.random.uniform(x0 - 10, x0 + 10)
    yt = np.random.uniform(y0 - 10, y0 + 10)
    start_episode(x0, y0, phi0, xt, yt)
    k = 0
    x_previous, y_previous = x, y
    records = []
    while not is_on_target(x, y, x_t, y_t):
        if max_calls is not None and len(records) == max_calls:
            return records, "max_calls"
        pre = (x, y, phi, v, t, optimal_criterion)
        coordinates = predictive_control(x, y, phi, v, x_t, y_t)
        records.append({"pre": pre, "ret": coordinates, "optimal_criterion": optimal_criterion})
        x, y, phi, v, beta = coordinates
        if x == x_previous and y == y_previous:
            k += 1
        if k == 2:
            return records, "recursive_error"
        x_previous, y_previous = x, y
    return records, "on_target"


def draw_starts(n, seed=None):
    """Start and target of n consecutive episodes exactly as the script's loop
    draws them (:235-239, five numpy uniforms per episode, one RNG stream)."""
    if seed is not None:
        np.random.seed(seed)
    out = []
    for _ in range(n):
        x0 = np.random.uniform(-10, 10)
        y0 = np.random.uniform(-10, 10)
        phi0 = np.random.uniform(-math.pi, math.pi)
        xt = np.random.uniform(x0 - 10, x0 + 10)
        yt = np.random.uniform(y0 - 10, y0 + 10)
        out.append((x0, y0, phi0, xt, yt))
    return out


class _Robot:
    """One episode's state (the script's module globals, per robot)."""

    def __init__(self, start):
        self.x_0, self.y_0, self.phi_0, self.x_t, self.y_t = start
        self.x, self.y, self.phi, self.v, self.beta = self.x_0, self.y_0, self.phi_0, 0, 0
        self.t = 0
        self.atan_t = float(np.arctan(self.x_t / self.y_t))
        self.crit = self._criterion0()
        self.stale = None            # optimal_trajectory[0][0] of the last winner
        self.k = 0
        self.prev = (self.x, self.y)
        self.records = []
        self.stop = None

    def _criterion0(self):
        # control_criterion([x_0, y_0, phi_0]) with this episode's globals (:82-86)
        angle = (np.arctan(self.x_t / self.y_t) - self.phi_0)
        dist_t = math.sqrt((self.x_t - self.x_0) ** 2 + (self.y_t - self.y_0) ** 2)
        return 10000 * dist_t + 10 * angle ** 2 + 100 * 1000 ** 2


def run_batched(starts, max_calls=None, integrator=None, chunk=256, stats=None):
    """The script's episode loop (:231-280) for len(starts) episodes at once,
    device-resident (mpc_fulltree_episodes_run, csrc/mpc_ftepisodes.h): one
    robot per episode; per call the robots still running are compacted and
    each one's S1^3 leaves spread over the whole GPU — the stop rules, t +=
    delta_t, the leaves against the robot's never-reset incumbent, its stale
    winner, the two-non-move stop — `chunk` calls per host call with no host
    step in between.  Returns
    [(records, stop)] per episode, as run_episode does (records rebuilt from
    the per-step log: pre = (x, y, phi, v, t, optimal_criterion) before the
    call, ret, optimal_criterion after it); raises the script's TypeError if an
    episode's first call finds no winner.  stats (optional dict) receives the
    lockstep-equivalent steps (the longest episode's calls) and the leaves."""
    from .abi import MPC_EP_ARRIVED, MPC_EP_BREAK, MPC_EP_NO_TRAJ
    robots = [_Robot(s) for s in starts]
    cap = min(chunk, max_calls) if max_calls else chunk
    eps_dev = device_ft_episodes(starts, max_calls, integrator, cap, robots)
    logs = [[] for _ in robots]
    while True:
        eps_dev.run(cap)
        for r, lg in enumerate(eps_dev.read_logs(first_step=[len(x) for x in logs])):
            logs[r].extend(lg[["x", "y", "phi", "v", "beta", "cost"]].tolist())
        calls, stop, leaves = eps_dev.read_progress()
        if (stop != 0).all():
            break
    if stats is not None:
        stats["steps"] = stats.get("steps", 0) + int(calls.max(initial=0))
        stats["leaves"] = stats.get("leaves", 0) + int(leaves.sum())
    out = []
    for r, lg, st in zip(robots, logs, stop):
        if st & MPC_EP_NO_TRAJ:
            raise TypeError("'int' object is not subscriptable")   # [0][0], as the script
        recs = []
        x, y, phi, v, t, crit = r.x, r.y, r.phi, r.v, r.t, r.crit
        for g in lg:
            ret = list(g[:5])                                 # x, y, phi, v, beta
            recs.append({"pre": (x, y, phi, v, t, crit), "ret": ret,
                         "optimal_criterion": g[5]})
            x, y, phi, v = ret[:4]
            t = t + delta_t
            crit = g[5]
        out.append((recs, "recursive_error" if st & MPC_EP_BREAK else
                    "on_target" if st & MPC_EP_ARRIVED else "max_calls"))
    return out


def device_ft_episodes(starts, max_calls=None, integrator=None, log_capacity=256, robots=None):
    """The device state of len(starts) full-tree episodes (episode.DeviceFtEpisodes)
    with the script's grids, constants and first incumbents: run_batched's
    engine, also driven directly by bench.py's workload G."""
    from .abi import MpcFulltreeEpisodeConfig
    from .episode import DeviceFtEpisodes
    eng, (vg, bg) = _device()
    integ = INTEGRATOR if integrator is None else integrator
    robots = robots or [_Robot(s) for s in starts]
    cfgs = [MpcFulltreeEpisodeConfig(float(r.x_0), float(r.y_0), float(r.phi_0), float(r.x_t),
                                     float(r.y_t), r.atan_t, float(r.crit), int(max_calls or 0), 0)
            for r in robots]
    return DeviceFtEpisodes(eng, cfgs, vg, bg, float(L), float(delta_t), float(eps), integ,
                            log_capacity=log_capacity)


def run_batched_lockstep(starts, max_calls=None, integrator=None):
    """The script's episode loop (:231-280) for len(starts) episodes at once:
    one robot per episode, all robots step in lockstep, and every MPC step of
    all still-running episodes is ONE batched full-tree launch
    (mpc_fulltree_argmin_batched) with the episode updates on the host (round
    3's driver, kept as the device-resident run_batched's cross-check).  Each
    robot keeps its own never-reset incumbent, stale winner and stop rule.
    Returns [(records, stop)] per episode, as run_episode does."""
    eng, (vg, bg) = _device()
    integ = INTEGRATOR if integrator is None else integrator
    robots = [_Robot(s) for s in starts]
    step = 0
    while True:
        live = []
        for r in robots:
            if r.stop is not None:
                continue
            if is_on_target_of(r):
                r.stop = "on_target"
            elif max_calls is not None and len(r.records) == max_calls:
                r.stop = "max_calls"
            else:
                live.append(r)
        if not live:
            break
        t_now = live[0].t + delta_t                       # lockstep: one window (:156)
        probs = (MpcFulltreeProblem * len(live))(*[
            MpcFulltreeProblem(float(r.x), float(r.y), float(r.phi), float(r.x_t),
                               float(r.y_t), float(r.x_0), float(r.y_0), r.atan_t, float(L),
                               t_now, t_now + delta_t) for r in live])
        pd = torch.frombuffer(bytearray(bytes(probs)), dtype=torch.uint8).to(eng.device)
        inc = torch.tensor([r.crit for r in live], dtype=torch.float64, device=eng.device)
        res = fulltree_results(fulltree_argmin_batched(eng, pd, inc, L, t_now, t_now + delta_t,
                                                       vg, bg, integ))
        for r, w in zip(live, res):
            pre = (r.x, r.y, r.phi, r.v, r.t, r.crit)
            r.t = t_now
            if w.found:
                r.crit = w.cost
                r.stale = [w.traj[0][0], w.traj[0][1], w.traj[0][2], w.v[0], w.beta[0]]
            if r.stale is None:
                raise TypeError("'int' object is not subscriptable")   # as the script
            coords = list(r.stale)
            r.records.append({"pre": pre, "ret": coords, "optimal_criterion": r.crit})
            r.x, r.y, r.phi, r.v, r.beta = coords
            if r.x == r.prev[0] and r.y == r.prev[1]:
                r.k += 1
            if r.k == 2:
                r.stop = "recursive_error"
            r.prev = (r.x, r.y)
        step += 1
    return [(r.records, r.stop) for r in robots]


def is_on_target_of(r):
    return (r.x_t - r.x) ** 2 + (r.y_t - r.y) ** 2 <= eps


# ----------------------------------------------------------------------------
# The script's episode loop over the tree expansion (SURVEY §8b "entry", Fact
# 2): at config.py's resolution the full tree above cannot run (S1^3 = 1.4e13
# leaves, MemoryError in the reference), so the named entry drives
# math_model_tree.py's MPC step instead — the acceleration-limited grid
# around the current (v, beta) (:239-256, <= 11 x 41 controls), N = 3 constant
# sequences, strict-< first minimum, the incumbent reset to sys.maxsize after
# every call (:428), the finishing logic m (:392-414) — inside the episode
# loop of run_math_model.py:231-280 (five uniform draws per episode,
# is_on_target, the two-non-move stop).  Per episode the script resets t, v
# and the incumbent (:233-234, :252); m, steps_for_slowing, optimal_trajectory
# and beta are reset too here, so that episodes are independent and can run
# side by side (the script leaks them from one episode into the next).

def _tree_globals(start):
    from . import math_model_tree as mmt
    x0, y0, phi0, xt, yt = start
    mmt.t = 0
    mmt.m = 0
    mmt.steps_for_slowing = 0
    mmt.x_t, mmt.y_t, mmt.x_0, mmt.y_0, mmt.phi_0 = xt, yt, x0, y0, phi0
    mmt.optimal_trajectory = [[[0]]]
    mmt.optimal_criterion = mmt.control_criterion([x0, y0, phi0])      # :252
    return mmt


def run_tree_episode(start, max_calls=None):
    """One episode of the script's loop (:231-280) whose MPC step is the drop-in
    math_model_tree.predictive_control (one C-ABI expansion per call).
    start = (x_0, y_0, phi_0, x_t, y_t) as draw_starts() draws them.
    Returns (list of returned [x, y, phi, v, beta], stop)."""
    mmt = _tree_globals(start)
    x0, y0, phi0, xt, yt = start
    x, y, phi, v, b = x0, y0, phi0, 0, 0
    k = 0
    x_previous, y_previous = x, y
    records = []
    while not is_on_target(x, y, xt, yt):
        if max_calls is not None and len(records) == max_calls:
            return records, "max_calls"
        c = mmt.predictive_control(x, y, phi, xt, yt, mmt.vector_of_velocities(v),
                                   mmt.vector_of_beta_angles(b), False)
        records.append(list(c))
        x, y, phi, v, b = c
        if x == x_previous and y == y_previous:
            k += 1
        if k == 2:
            return records, "recursive_error"
        x_previous, y_previous = x, y
    return records, "on_target"


def run_tree_batched(starts, max_calls=None, integrator="qk21", engine=None, stats=None,
                     chunk=1024):
    """The tree-expansion episode loop for len(starts) episodes at once, one
    robot per episode, device-resident (episode.DeviceEpisodes,
    mpc_episodes_run): each robot is one block that runs its episode's MPC
    steps back to back — its grid around its own (v, beta), the reference's
    enumeration, the expansion, the winner, the finishing logic m, the two-
    non-move stop and the on-target test, all on the device — `chunk` steps
    per launch, the log read back once per launch.  Returns [(records, stop)]
    per episode, as run_tree_episode returns them (the script's TypeError if
    an episode's first call finds no winner).  stats (optional dict) receives
    the lockstep-equivalent steps (the longest episode's calls) and the
    candidates rolled out (each call's |V| x |B|)."""
    import numpy as np
    from .abi import MPC_EP_ARRIVED, MPC_EP_BREAK
    from .episode import DeviceEpisodes, tree_episode_config
    eng = engine or _device()[0]
    R = len(starts)
    if max_calls == 0:
        return [([], "on_target" if is_on_target(s[0], s[1], s[3], s[4]) else "max_calls")
                for s in starts]
    cap = min(chunk, max_calls) if max_calls else chunk
    eps = DeviceEpisodes(eng, [tree_episode_config(s, max_calls) for s in starts], 3, integrator,
                         log_capacity=cap)
    records = [[] for _ in range(R)]
    found_any = np.zeros(R, dtype=bool)
    while True:
        eps.run(cap)
        logs = eps.read_logs(first_step=[len(r) for r in records])
        calls, stop, cands = eps.read_progress()
        for r, lg in enumerate(logs):
            if len(lg) == 0:
                continue
            f = lg["found"] != 0
            if not found_any[r] and not f[0]:
                raise TypeError("'int' object is not subscriptable")   # [[[0]]], as the script
            found_any[r] |= bool(f.any())
            records[r].extend(np.stack([lg["x"], lg["y"], lg["phi"], lg["v"], lg["beta"]],
                                       axis=1).tolist())
        if (stop != 0).all():
            break
    if stats is not None:
        stats["steps"] = stats.get("steps", 0) + int(calls.max(initial=0))
        stats["candidates"] = stats.get("candidates", 0) + int(cands.sum())
    names = []
    for st in stop:
        names.append("recursive_error" if st & MPC_EP_BREAK else
                     "on_target" if st & MPC_EP_ARRIVED else "max_calls")
    return [(records[r], names[r]) for r in range(R)]


__all__ = ["configure", "shard_over", "draw_starts", "run_batched", "run_batched_lockstep",
           "is_on_target",
           "get_distance_from_line", "get_distance_from_target", "saturation", "control_criterion",
           "predictive_control", "start_episode", "run_episode", "prediction_horizon",
           "run_tree_episode", "run_tree_batched"]
