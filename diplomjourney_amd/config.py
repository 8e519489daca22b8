"""Model constants for the MPC expansion — the reference's config.py surface.

The reference imports these 16 names by name (math_model_tree.py:13-14,
run_math_model.py:9); values are those of its config.py:3-28.  Integers stay
integers (v_max, x_0, y_0, phi_0, x_t, y_t) because Python int/float mixing is
part of the reference arithmetic (e.g. `10000 * 1000 ** 2` in the cost).
"""
from math import radians as _rad

# vehicle: distance between axles [m]; steering/velocity model of v_phi (:77-78)
L = 0.5

# control period [s]: integration window of every quad() call
delta_t = 0.05

# steering angle beta: bound, grid step, max rate [rad, rad, rad/s]
beta_max = _rad(60)
delta_beta = _rad(1)
beta_acc_max = _rad(400)

# speed v: bounds, grid step [m/s], max acceleration [m/s^2]
v_max = 1
v_min = 0.4
delta_v = 0.005
v_acc_max = 0.5

# arrival tolerance on the squared distance, and steering-bound margin
eps = 0.001
eps_beta = _rad(5)

# start pose (also the origin of the reference line used by the cost)
x_0 = 0
y_0 = 0
phi_0 = 0

# operator target
x_t = 1
y_t = 5

__all__ = ["L", "delta_t", "beta_max", "delta_beta", "beta_acc_max", "v_max", "v_min",
           "delta_v", "v_acc_max", "eps", "eps_beta", "x_0", "y_0", "phi_0", "x_t", "y_t"]
