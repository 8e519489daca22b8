"""MPC episode at scale: the reference's math_mpc loop (math_model_tree.py:515-635)
driving sampled candidate sets of arbitrary size and horizon on one or more
GPUs.

Per MPC step (one `Episode.step()`):
  1. host: the reference's acceleration-limited grid around the current
     (v, beta) (:239-256), slow-down override (:312-316)            <= 451 entries
  2. device: k_sample_controls -> fp64 SoA [N, C_local] in HBM
     (candidates 0..|grid|-1 are the reference's constant sequences)
  3. device: k_rollout_argmin (the HBM-streaming kernel) + k_finalize
  4. multi-GPU: all_gather of the 808-B winner records + k_select_winner
  5. one 808-B device->host read; host applies the reference's finishing
     logic (:366-429) and operator events (p = 60 / 90 / 110, :564-569)
The incumbent is sys.maxsize after the first call, as in the reference
(:428); the episode restarts from the start pose when the target is reached.
"""
import math
import sys
import time

import torch

from . import math_model_tree as mmt
from .abi import make_problem
from .distributed import exchange_winner, shard_range


class Episode:
    def __init__(self, engine, n_cand_total, n_steps, rank=0, world=1, seed=20261015,
                 integrator="rect", group=None, start=(0.0, 0.0, 0.0, 0.0, 0.0), target=(2, 3)):
        self.eng = engine
        self.n_total = int(n_cand_total)
        self.n_steps = int(n_steps)
        self.rank, self.world, self.group = rank, world, group
        self.lo, self.hi = shard_range(self.n_total, rank, world)
        self.n_local = self.hi - self.lo
        self.seed = seed
        self.integrator = integrator
        self.start, self.target = start, target
        dev = engine.device
        self.v_sc = torch.empty((self.n_steps, self.n_local), dtype=torch.float64, device=dev)
        self.b_sc = torch.empty_like(self.v_sc)
        self._grid_host = torch.empty(2 * 451, dtype=torch.float64).pin_memory()
        self._grid_dev = torch.empty(2 * 451, dtype=torch.float64, device=dev)
        self.kernel_ms = []          # device time of the streaming kernel, per step
        self.step_ms = []            # host wall time per MPC step
        self._ev = None
        self.reset()

    # -- episode state (reference globals of math_mpc) -------------------------
    def reset(self):
        x, y, phi, v, beta = self.start
        self.x, self.y, self.phi, self.v, self.beta = x, y, phi, v, beta
        self.x_t, self.y_t = self.target
        self.x_0, self.y_0 = x, y
        self.t = 0.0
        self.p = 1
        self.m = 0
        self.steps_for_slowing = 0
        self.episodes = getattr(self, "episodes", 0) + 1
        self.incumbent = self._criterion0()

    def _criterion0(self):
        saved = (mmt.x_t, mmt.y_t, mmt.x_0, mmt.y_0)
        mmt.x_t, mmt.y_t, mmt.x_0, mmt.y_0 = self.x_t, self.y_t, self.x_0, self.y_0
        c = mmt.control_criterion([self.x_0, self.y_0, 0.0])
        mmt.x_t, mmt.y_t, mmt.x_0, mmt.y_0 = saved
        return c

    # -- one MPC step -------------------------------------------------------------
    def _grids(self):
        V = mmt.vector_of_velocities(self.v)
        B = mmt.vector_of_beta_angles(self.beta)
        if self.steps_for_slowing > 0 and V:
            vel = min(V) if min(V) > mmt.v_min else mmt.v_min
            V = [vel] * len(V)
        return V, B

    def step(self, time_kernel=False):
        t0 = time.perf_counter()
        V, B = self._grids()
        nv, nb = len(V), len(B)
        self._grid_host[:nv] = torch.tensor(V, dtype=torch.float64)
        self._grid_host[nv:nv + nb] = torch.tensor(B, dtype=torch.float64)
        self._grid_dev[:nv + nb].copy_(self._grid_host[:nv + nb], non_blocking=True)
        self.t += mmt.delta_t
        seed = (self.seed + 0x9E3779B9 * (self.p + 1000 * self.episodes)) & 0xFFFFFFFFFFFFFFFF
        self.eng.sample_controls(self._grid_dev[:nv], self._grid_dev[nv:nv + nb], self.n_local,
                                 self.n_steps, seed, index_base=self.lo, v_out=self.v_sc,
                                 beta_out=self.b_sc)
        prob = make_problem(self.x, self.y, self.phi, self.x_t, self.y_t, self.x_0, self.y_0,
                            mmt.L, self.t, self.t + mmt.delta_t)
        if time_kernel:
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
        self.eng.partials(prob, self.v_sc, self.b_sc, self.integrator)
        if time_kernel:
            e1.record()
        out = self.eng.finalize(prob, self.v_sc, self.b_sc, index_base=self.lo,
                                incumbent=self.incumbent, integrator=self.integrator,
                                out=self.eng.result)
        if self.world > 1:
            exchange_winner(self.eng, out, incumbent=self.incumbent, group=self.group)
        res = self.eng.fetch()
        if time_kernel:
            self.kernel_ms.append(e0.elapsed_time(e1))
        self._advance(res)
        self.step_ms.append((time.perf_counter() - t0) * 1e3)
        return res

    def _advance(self, res):
        """Reference post-processing + episode bookkeeping (:351-429, :542-579)."""
        self.steps_for_slowing -= 1
        self.incumbent = float(sys.maxsize)
        if not res.found:
            # nothing beat the incumbent: keep the pose (stale trajectory)
            return
        traj = res.trajectory()
        k = 0
        if self.m == 2:
            k = 2
        elif self.m == 1:
            k = 1
            self.m += 1
        elif mmt.is_on_target(traj[min(2, self.n_steps - 1)][0],
                              traj[min(2, self.n_steps - 1)][1], self.x_t, self.y_t)[0]:
            self.m += 1
        k = min(k, self.n_steps - 1)
        self.x, self.y, self.phi = traj[k]
        self.v, self.beta = res.v, res.beta
        if self.p == 60:
            self._turn(-1)
        if self.p == 90:
            self._turn(+1)
        if self.p == 110:
            self._new_target(2, 3)
        self.p += 1
        if mmt.is_on_target(self.x, self.y, self.x_t, self.y_t)[0] or self.p > 400:
            self.reset()

    def _new_target(self, tx, ty):
        self.x_t, self.y_t = tx, ty
        self.x_0, self.y_0 = self.x, self.y
        self.steps_for_slowing = 10          # slow_down(radians(30)), :128

    def _turn(self, sign):
        tx, ty = mmt._turn_target(self.x, self.y, self.phi, 2, sign)
        self._new_target(tx, ty)
        self.steps_for_slowing = 20          # slow_down(radians(90)), :175/:213


def percentile(xs, q):
    if not xs:
        return math.nan
    s = sorted(xs)
    i = min(len(s) - 1, max(0, int(round(q / 100.0 * (len(s) - 1)))))
    return s[i]
