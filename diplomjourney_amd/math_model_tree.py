"""Host side of the MPC step, with the reference's call surface and globals.

Mirrors ShittyWizard/DiplomJourney's math_model_tree.py: the same function
names, argument meaning, module-global state and return values, so code that
drives the reference's `predictive_control` (math_model_tree.py:278) or
`math_mpc` (:515) runs unchanged against this module.  What changes is where
the work happens:

* predictive_control (:278-496): the three hard-coded layer loops over
  |V|*|B| candidates (:308-360) and the CoordinateTree fill become ONE launch
  of the HIP expansion kernel (libmpc_rollout.so, mpc_rollout_argmin) over an
  fp64 SoA candidate set in HBM, with the tree's node states written by the
  kernel; one 808-byte result record comes back per MPC step.
* everything else (grid generation :239-256, the finishing logic :366-429,
  operator events :118-226, the episode loop :515-635) is the reference's host
  logic, restated here in plain Python.

Plotting (:719-941) and the print-outs are not reproduced (set VERBOSE = True
for the reference's progress lines).  There is no CPU fallback for the
expansion: without a GPU and the built library, predictive_control raises.
"""
import math
import sys
import time

import numpy as np
import torch

from . import config as _cfg
from .abi import make_problem
from .CoordinateTree import CoordinateTree

L = _cfg.L
beta_acc_max = _cfg.beta_acc_max
beta_max = _cfg.beta_max
delta_beta = _cfg.delta_beta
delta_t = _cfg.delta_t
delta_v = _cfg.delta_v
eps = _cfg.eps
v_acc_max = _cfg.v_acc_max
v_max = _cfg.v_max
v_min = _cfg.v_min
eps_beta = _cfg.eps_beta

# The reference's `from scipy import *` (:11) binds `random` to numpy.random
# (SURVEY Appendix A): its perturbations draw from numpy's global RNG.
random = np.random

VERBOSE = False
# Integration rule of the device kernel: "qk21" reproduces sp.quad bit for bit
# on a constant integrand (the reference's arithmetic); "rect" evaluates the same
# integrals directly (h*f, positions with one fused rounding; mpc_device.h).
INTEGRATOR = "qk21"

# Prediction horizon * delta_t = 0.15 s (:27)
prediction_horizon = 3

# Radius of U-turn (:44)
radius_u_turn = L / math.sin(beta_max)

_engine = None


def _say(*a):
    if VERBOSE:
        print(*a)


def engine():
    """The per-process device engine (created on first use)."""
    global _engine
    if _engine is None:
        from .expansion import Expansion
        _engine = Expansion()
    return _engine


def reset_state():
    """Module state as the reference sets it at import time (:19-24, :638-717)."""
    g = globals()
    g.update(beta=0, v=0, phi=_cfg.phi_0, x=_cfg.x_0, y=_cfg.y_0,
             x_0=_cfg.x_0, y_0=_cfg.y_0, phi_0=_cfg.phi_0, x_t=_cfg.x_t, y_t=_cfg.y_t,
             t=0, dt=delta_t, p=1, recursive=False, need_scatter=False,
             time_arr_for_plotting=[0], actual_time_arr_for_plotting=[0],
             optimal_trajectory=[[[0]]],
             result_trajectory_phi=[_cfg.phi_0], actual_result_trajectory_phi=[_cfg.phi_0],
             result_trajectory_x=[_cfg.x_0], actual_result_trajectory_x=[_cfg.x_0],
             result_trajectory_y=[_cfg.y_0], actual_result_trajectory_y=[_cfg.y_0],
             result_x_velocity=[0], result_x_acceleration=[0],
             result_y_velocity=[0], result_y_acceleration=[0],
             result_trajectory_v=[0], actual_result_trajectory_v=[0],
             result_trajectory_beta=[0], actual_result_trajectory_beta=[0],
             result_trajectory_angle_speed=[0], actual_result_trajectory_angle_speed=[0],
             result_v=0, result_beta=0, m=0, steps_for_slowing=0,
             last_tree=None, last_result=None)
    for name in ("predicted_trajectory", "actual_predicted_trajectory"):
        for ax in ("x", "y", "phi"):
            for k in range(3):
                g[f"{name}_{ax}_anim{k}"] = []
    g["optimal_criterion"] = control_criterion([x_0, y_0, phi_0])


# ----------------------------------------------------------------------------
# Scalar helpers (host).  Same arithmetic as the reference's :48-87.
def is_on_target(actual_x, actual_y, target_x, target_y):
    d2 = (target_x - actual_x) ** 2 + (target_y - actual_y) ** 2
    return [d2 <= eps, d2]


def get_distance_from_line(x_a, y_a):
    """Squared distance to the line origin->target; 1000**2 at the origin (:56-62)."""
    if x_a == x_0 and y_a == y_0:
        dist = 1000
    else:
        dist = (abs((y_t - y_0) * x_a - (x_t - x_0) * y_a + x_t * y_0 - y_t * x_0)
                / math.sqrt((y_t - y_0) ** 2 + (x_t - x_0) ** 2))
    return dist ** 2


def get_distance_from_target(x_a, y_a):
    return math.sqrt((x_t - x_a) ** 2 + (y_t - y_a) ** 2)


def control_criterion(predicted_coordinates):
    """Host evaluation of the cost for ONE state (used for the first incumbent,
    :676); the per-candidate costs are computed on the GPU."""
    return (10000 * get_distance_from_target(predicted_coordinates[0], predicted_coordinates[1])
            + 10000 * get_distance_from_line(predicted_coordinates[0], predicted_coordinates[1]))


# ----------------------------------------------------------------------------
# Acceleration-limited control grids (:239-256).
def vector_of_velocities(actual_velocity):
    ratio = (v_acc_max * delta_t) / delta_v
    out = []
    for i in range(1 + 2 * int(ratio)):
        cand = actual_velocity + delta_v * (i - ratio)
        if (not cand < 0) and cand < v_max:
            out.append(cand)
    return out


def vector_of_beta_angles(actual_beta):
    ratio = (math.degrees(beta_acc_max) * delta_t) / math.degrees(delta_beta)
    bound = beta_max + math.radians(eps_beta)
    out = []
    for i in range(1 + 2 * int(ratio)):
        cand = actual_beta + delta_beta * (i - ratio)
        if abs(cand) <= bound:
            out.append(cand)
    return out


# ----------------------------------------------------------------------------
# Operator events (:118-226).
def plot_from_actual_to_target(initial_x, initial_y, initial_phi, target_x, target_y):
    """Plotting hook (:132-139); figures are out of scope."""


def slow_down(delta_teta):
    global steps_for_slowing
    a = abs(delta_teta)
    if a < math.radians(10):
        steps_for_slowing = 0
    elif a <= math.radians(45):
        steps_for_slowing = 10
    elif a <= math.radians(90):
        steps_for_slowing = 20


def new_target(actual_x, actual_y, actual_phi, target_x, target_y, actual_velocity):
    global x_t, y_t, x_0, y_0, phi_0
    _say("Previous target: " + str(x_t) + " " + str(y_t))
    x_t, y_t = target_x, target_y
    x_0, y_0, phi_0 = actual_x, actual_y, actual_phi
    plot_from_actual_to_target(actual_x, actual_y, actual_phi, target_x, target_y)
    slow_down(math.radians(30))
    _say("New target: " + str(x_t) + " " + str(y_t))


def _turn_target(actual_x, actual_y, actual_phi, distance, sign):
    """Target of a U-turn (:142-215).  sign = +1 turn_left, -1 turn_right.
    The reference's four heading sectors are kept with their expressions."""
    c, s = math.cos, math.sin
    R = radius_u_turn
    if math.pi / 2 <= actual_phi <= 3 * math.pi / 2:
        if actual_phi <= math.pi:
            tp = actual_phi - math.pi / 2
            tx = actual_x - sign * distance * c(tp) - R * s(tp)
            ty = actual_y - sign * distance * s(tp) + R * c(tp)
        else:
            tp = actual_phi - math.pi
            tx = actual_x + sign * distance * s(tp) - R * c(tp)
            ty = actual_y - sign * distance * c(tp) - R * s(tp)
    else:
        if actual_phi <= 2 * math.pi:
            tp = actual_phi - 3 * math.pi / 2
            tx = actual_x + sign * distance * c(tp) + R * s(tp)
            ty = actual_y + sign * distance * s(tp) - R * c(tp)
        else:
            tp = actual_phi
            tx = actual_x - sign * distance * s(tp) + R * c(tp)
            ty = actual_y + sign * distance * c(tp) + R * s(tp)
    return tx, ty


def turn_left(actual_x, actual_y, actual_phi, distance, actual_velocity):
    tx, ty = _turn_target(actual_x, actual_y, actual_phi, distance, +1)
    new_target(actual_x, actual_y, actual_phi, tx, ty, actual_velocity)
    slow_down(math.radians(90))
    _say("Turning left...")


def turn_right(actual_x, actual_y, actual_phi, distance, actual_velocity):
    tx, ty = _turn_target(actual_x, actual_y, actual_phi, distance, -1)
    new_target(actual_x, actual_y, actual_phi, tx, ty, actual_velocity)
    slow_down(math.radians(90))
    _say("Turning right...")


def get_actual_velocity(velocity_ref):
    """Plant perturbation of the 'actual' run (:259-267), numpy global RNG."""
    if random.random() < 0.7:
        if velocity_ref < 0.4:
            return velocity_ref + (random.randint(0, 5) / 1000)
        return velocity_ref + (random.randint(-100, 10) / 1000)
    return velocity_ref


def get_actual_beta_angle(beta_ref):
    if random.random() < 0.7:
        return beta_ref + math.radians(random.randint(-5, 5))
    return beta_ref


# ----------------------------------------------------------------------------
# The MPC step.
def candidate_controls(vector_v, vector_beta, n_steps, device):
    """fp64 SoA [n_steps, |V|*|B|] of the reference's enumeration: candidate
    k = a*|B| + b holds (V[a], B[b]) at every step (:311-317, SURVEY Fact 1)."""
    V = torch.tensor(vector_v, dtype=torch.float64)
    B = torch.tensor(vector_beta, dtype=torch.float64)
    vv = V.repeat_interleave(len(vector_beta))
    bb = B.repeat(len(vector_v))
    v_sc = vv.unsqueeze(0).expand(n_steps, -1).contiguous().to(device, non_blocking=True)
    b_sc = bb.unsqueeze(0).expand(n_steps, -1).contiguous().to(device, non_blocking=True)
    return v_sc, b_sc


def _finish(isActual, ot):
    """Post-processing of :366-429 (model run) / :430-496 (actual run)."""
    global m, optimal_criterion
    px = [ot[0][0], ot[1][0], ot[2][0]]
    py = [ot[0][1], ot[1][1], ot[2][1]]
    pphi = [ot[0][2], ot[1][2], ot[2][2]]
    pre = "actual_predicted_trajectory" if isActual else "predicted_trajectory"
    g = globals()
    for k in range(3):
        g[f"{pre}_x_anim{k}"].append(px[k])
        g[f"{pre}_y_anim{k}"].append(py[k])
        g[f"{pre}_phi_anim{k}"].append(pphi[k])
    rx, ry, rphi = px[0], py[0], pphi[0]
    if m == 2:
        rx, ry, rphi = px[2], py[2], pphi[2]
    elif m == 1:
        rx, ry, rphi = px[1], py[1], pphi[1]
        m += 1
    elif is_on_target(px[2], py[2], x_t, y_t)[0]:
        m += 1
    if not isActual:
        result_trajectory_x.append(rx)
        result_trajectory_y.append(ry)
        result_trajectory_phi.append(rphi)
        result_trajectory_v.append(result_v)
        result_trajectory_beta.append(result_beta)
        result_trajectory_angle_speed.append((result_v / L) * math.tan(result_beta))
    else:
        actual_result_trajectory_x.append(rx)
        actual_result_trajectory_y.append(ry)
        actual_result_trajectory_phi.append(rphi)
    _say("Now I'm here - x : " + str(rx) + " y: " + str(ry) + " v: " + str(result_v)
         + " beta: " + str(math.degrees(result_beta)))
    optimal_criterion = sys.maxsize
    return [rx, ry, rphi, result_v, result_beta]


def predictive_control(_initial_x, _initial_y, _initial_phi, _target_x, _target_y, _vector_v,
                       _vector_beta, isActual):
    """One MPC step (:278-496).  Like the reference, `_target_x/_target_y` are
    ignored: the cost reads the globals x_t, y_t, x_0, y_0."""
    global optimal_trajectory, optimal_criterion, t, m, result_v, result_beta
    global steps_for_slowing, last_tree, last_result
    eng = engine()
    size_max_1 = len(_vector_beta) * len(_vector_v)
    global_coordinates = CoordinateTree(size_max_1, prediction_horizon, device=eng.device)

    t += delta_t
    (actual_time_arr_for_plotting if isActual else time_arr_for_plotting).append(t)
    start = time.time()

    V = list(_vector_v)
    if steps_for_slowing > 0 and V:
        vmin_v = np.min(V)
        vel = vmin_v if vmin_v > v_min else v_min           # :312-316
        V = [vel] * len(V)
    if size_max_1 > 0:
        v_sc, b_sc = candidate_controls(V, list(_vector_beta), prediction_horizon, eng.device)
        problem = make_problem(_initial_x, _initial_y, _initial_phi, x_t, y_t, x_0, y_0, L,
                               t, t + delta_t)
        eng.rollout_argmin(problem, v_sc, b_sc, incumbent=optimal_criterion,
                           integrator=INTEGRATOR, states=global_coordinates.states)
        global_coordinates.controls[0].copy_(v_sc[0])
        global_coordinates.controls[1].copy_(b_sc[0])
        res = eng.fetch()
        global_coordinates.mark_filled()
        if res.found:                                                   # :351-359
            ctl = [V[res.index // len(_vector_beta)], _vector_beta[res.index % len(_vector_beta)]]
            traj = res.trajectory()
            optimal_trajectory = [[traj[0] + ctl, traj[1] + ctl, traj[2] + ctl]]
            result_v, result_beta = ctl
            optimal_criterion = res.cost
        last_result = res
    last_tree = global_coordinates
    steps_for_slowing -= 1
    _say("Third layer done.Time = " + str(time.time() - start))
    return _finish(isActual, optimal_trajectory[0])


# ----------------------------------------------------------------------------
# Episode loop (:515-635).
def math_mpc(initial_coordinates, target_coordinates, isActual, on_step=None):
    global x, y, phi, x_t, y_t, v, beta, recursive, p, t
    p = 1
    t = 0
    x_t, y_t = target_coordinates[0], target_coordinates[1]
    recursive = False
    plot_from_actual_to_target(x_0, y_0, phi_0, x_t, y_t)
    if not isActual:
        x, y, phi = initial_coordinates[0], initial_coordinates[1], initial_coordinates[2]
        v = initial_coordinates[3]
        beta = initial_coordinates[4]
        x_prev, y_prev = x, y
        while not is_on_target(x, y, x_t, y_t)[0]:
            prev_v = v
            coords = predictive_control(x, y, phi, x_t, y_t, vector_of_velocities(v),
                                        vector_of_beta_angles(beta), isActual)
            x, y, phi, v, beta = coords
            if on_step:
                on_step(p, coords)
            if recursive:
                _say("Recursive error.")
                break
            elif x == x_prev and y == y_prev:
                recursive = True
            if p == 60:
                turn_right(x, y, phi, 2, v)
            if p == 90:
                turn_left(x, y, phi, 2, v)
            if p == 110:
                new_target(x, y, phi, 2, 3, v)
            x_prev, y_prev = x, y
            p += 1
            result_x_velocity.append(v * math.cos(phi))
            result_x_acceleration.append(((v - prev_v) / delta_t) * math.cos(phi))
            result_y_velocity.append(v * math.sin(phi))
            result_y_acceleration.append(((v - prev_v) / delta_t) * math.sin(phi))
    else:
        ax, ay, aphi = initial_coordinates[0], initial_coordinates[1], initial_coordinates[2]
        av = initial_coordinates[3]
        abeta = initial_coordinates[4]
        x_prev, y_prev = ax, ay
        while not is_on_target(ax, ay, x_t, y_t)[0]:
            coords = predictive_control(ax, ay, aphi, x_t, y_t, vector_of_velocities(av),
                                        vector_of_beta_angles(abeta), isActual)
            ax, ay, aphi = coords[0], coords[1], coords[2]
            av = get_actual_velocity(coords[3])
            abeta = get_actual_beta_angle(coords[4])
            if on_step:
                on_step(p, coords)
            actual_result_trajectory_v.append(av)
            actual_result_trajectory_beta.append(abeta)
            actual_result_trajectory_angle_speed.append((av / L) * math.tan(abeta))
            if recursive:
                _say("Recursive error.")
                break
            elif ax == x_prev and ay == y_prev:
                recursive = True
            if p == 1:
                new_target(ax, ay, aphi, 2, 3, av)
            if p == 60:
                turn_right(ax, ay, aphi, 2, av)
            if p == 90:
                turn_left(ax, ay, aphi, 2, av)
            if p == 110:
                new_target(ax, ay, aphi, 2, 3, av)
            x_prev, y_prev = ax, ay
            p += 1
    t = 0


def run_reference_scenario(seed=0, on_step=None):
    """The reference's MODELLING block (:736-738): model run, then the actual
    run with numpy's RNG seeded (the reference leaves it unseeded)."""
    reset_state()
    math_mpc([0, 0, 0, 0, 0], [2, 3], False, on_step=on_step)
    global m
    m = 0
    np.random.seed(seed)
    math_mpc([0, 0, 0, 0, 0], [2, 3], True, on_step=on_step)


reset_state()
