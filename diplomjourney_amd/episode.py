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
     logic (:366-429) — on the stale optimal_trajectory when no candidate
     beat the incumbent — the stuck detector (:559-563) and the operator
     events (p = 60 / 90 / 110, :564-569)
The incumbent is sys.maxsize after the first call, as in the reference
(:428); an episode that ends (on target, :542, or "Recursive error",
:559-561) restarts from the start pose.
"""
import ctypes
import math
import sys
import time
import weakref

import torch

from . import math_model_tree as mmt
from .abi import (CANDIDATE_BYTES, IPC_HANDLE_BYTES, LOG_BYTES, MPC_EP_ARRIVED, MPC_EP_BREAK, MPC_EP_EVENT,
                  MPC_EP_LIMIT, MPC_EP_STALE, MPC_EP_STUCK, RESULT_BYTES, MpcEpisodeConfig,
                  MpcEpisodeLog, make_problem)
from .distributed import exchange_winner, gather_bytes, gather_into, gather_results, shard_range
from . import native

CHAIN_ERRORS = {
    1: "a chained launch's tile blocks timed out waiting for block 0's published constants "
       "(the step was scored on speculated constants)",
    2: "the state was reset with another wheelbase form (power of two or not) than the "
       "launch's cfg",
    3: "an exchange launch's block 0 timed out collecting its tile records (this rank's "
       "candidate dropped out of the global arg-min)",
    4: "an overlapped exchange launch's block 0 timed out waiting for the all_gather's mark "
       "(the collective could not run beside the launch: the step was not completed)",
    5: "a P2P exchange launch's block 0 timed out waiting for the ranks' candidates in its "
       "mailbox (a peer did not run the same step: the step was not completed)",
    6: "a one-GPU chained step's early publication of the next step's constants disagreed "
       "with its update (a self-check: never expected)",
}


class ChainError(RuntimeError):
    """A device-resident episode's bounded wait failed (EpisodeState::chain_error)."""

    def __init__(self, code):
        self.code = int(code)
        super().__init__(f"chain_error {self.code}: {CHAIN_ERRORS.get(self.code, 'unknown')}")


class Episode:
    def __init__(self, engine, n_cand_total, n_steps, rank=0, world=1, seed=20261015,
                 integrator="rect", group=None, start=(0.0, 0.0, 0.0, 0.0, 0.0), target=(2, 3),
                 max_steps=0):
        self.eng = engine
        self.max_steps = int(max_steps)
        # module globals of the reference that outlive an episode: the last
        # winner's layer states, result_v, result_beta (None: the initial
        # [[[0]]], which has no layer states)
        self.ot = None
        self.last_log = None
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
        self.x_prev, self.y_prev = x, y
        self.recursive = False
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

    def step(self, time_kernel=False, events=None):
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
        if time_kernel and events is None:
            events = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        if events:
            events[0].record()
        self.eng.partials(prob, self.v_sc, self.b_sc, self.integrator)
        if events:
            events[1].record()
        out = self.eng.finalize(prob, self.v_sc, self.b_sc, index_base=self.lo,
                                incumbent=self.incumbent, integrator=self.integrator,
                                out=self.eng.result)
        if self.world > 1:
            exchange_winner(self.eng, out, incumbent=self.incumbent, group=self.group)
        res = self.eng.fetch()
        if time_kernel:
            self.kernel_ms.append(events[0].elapsed_time(events[1]))
        self._advance(res)
        self.step_ms.append((time.perf_counter() - t0) * 1e3)
        return res

    def _advance(self, res):
        """The rest of math_mpc's loop body (:542-574 with :351-429); the same
        update as the device's episode_advance (csrc/mpc_episode.h)."""
        self.steps_for_slowing -= 1
        self.incumbent = float(sys.maxsize)
        step_p, status = self.p, 0
        if res.found:
            traj = res.trajectory()
            last = self.n_steps - 1
            self.ot = [list(traj[min(k, last)]) for k in range(3)]
            self.ot_v, self.ot_beta = res.v, res.beta
        else:
            status |= MPC_EP_STALE
            if self.ot is None:           # [[[0]]] has no layers: stay at the pose
                self.ot = [[self.x, self.y, self.phi] for _ in range(3)]
                self.ot_v, self.ot_beta = self.v, self.beta
        k = 0
        if self.m == 2:
            k = 2
        elif self.m == 1:
            k = 1
            self.m += 1
        elif mmt.is_on_target(self.ot[2][0], self.ot[2][1], self.x_t, self.y_t)[0]:
            self.m += 1
        self.x, self.y, self.phi = self.ot[k]
        self.v, self.beta = self.ot_v, self.ot_beta
        ended = False
        if self.recursive:                # "Recursive error." (:559-561)
            status |= MPC_EP_BREAK
            ended = True
        else:
            if self.x == self.x_prev and self.y == self.y_prev:
                self.recursive = True
                status |= MPC_EP_STUCK
            if self.p == 60:
                self._turn(-1)
                status |= MPC_EP_EVENT
            if self.p == 90:
                self._turn(+1)
                status |= MPC_EP_EVENT
            if self.p == 110:
                self._new_target(2, 3)
                status |= MPC_EP_EVENT
            self.x_prev, self.y_prev = self.x, self.y
            self.p += 1
            if mmt.is_on_target(self.x, self.y, self.x_t, self.y_t)[0]:
                status |= MPC_EP_ARRIVED
                ended = True
            elif self.max_steps > 0 and self.p > self.max_steps:
                status |= MPC_EP_LIMIT
                ended = True
        self.last_log = (res.index if res.found else -1, res.cost, step_p, self.x, self.y,
                         self.phi, self.v, self.beta, int(bool(res.found)), status)
        if ended:
            self.reset()

    def _new_target(self, tx, ty):
        self.x_t, self.y_t = tx, ty
        self.x_0, self.y_0 = self.x, self.y
        self.steps_for_slowing = 10          # slow_down(radians(30)), :128

    def _turn(self, sign):
        tx, ty = mmt._turn_target(self.x, self.y, self.phi, 2, sign)
        self._new_target(tx, ty)
        self.steps_for_slowing = 20          # slow_down(radians(90)), :175/:213


def reference_episode_config(start=(0.0, 0.0, 0.0, 0.0, 0.0), target=(2, 3), seed=20261015,
                             max_steps=0, incumbent0=0.0, enumerate=False):
    """mpc_episode_config_t with the reference's constants and expressions
    (config.py; grid ratios as math_model_tree.py:241-253 computes them; the
    operator schedule of :564-569; slow_down bands of :219-226).  max_steps 0:
    no step limit (the reference's loop runs until on target or stuck);
    incumbent0 0: the first incumbent from the episode's target (the
    reference's, 10000050990.195135, is config.py's target's, :676);
    enumerate: sampled steps hold exactly the step's |V|*|B| constant
    sequences (the reference's candidate set), the rest padding."""
    c = mmt._cfg
    return MpcEpisodeConfig(
        start_x=start[0], start_y=start[1], start_phi=start[2], start_v=start[3],
        start_beta=start[4], target_x=target[0], target_y=target[1],
        L=c.L, delta_t=c.delta_t, eps=c.eps, v_max=c.v_max, v_min=c.v_min, delta_v=c.delta_v,
        ratio_v=(c.v_acc_max * c.delta_t) / c.delta_v, delta_beta=c.delta_beta,
        ratio_beta=(math.degrees(c.beta_acc_max) * c.delta_t) / math.degrees(c.delta_beta),
        beta_bound=c.beta_max + math.radians(c.eps_beta), radius_u_turn=mmt.radius_u_turn,
        turn_distance=2.0, event_target_x=2.0, event_target_y=3.0,
        p_turn_right=60, p_turn_left=90, p_new_target=110, slow_new_target=10, slow_turn=20,
        max_steps=max_steps, incumbent0=incumbent0, enumerate=int(bool(enumerate)), seed=seed)


def logged_step_problems(log, cfg):
    """The problem and incumbent every logged step of a device episode was
    solved on, rebuilt on the host from the log records before it — the
    bookkeeping of episode_advance (csrc/mpc_episode.h) / Episode._advance:
    t += delta_t per step (math_model_tree.py:302), the pose of the previous
    record, the incumbent (the episode's first from cfg.incumbent0 or the
    criterion of the line origin, :676; then float(sys.maxsize), :428), the
    operator events at cfg.p_turn_right / p_turn_left / p_new_target
    (:564-569: new target, line origin at the pose) and a restart after a step
    that ended the episode (ARRIVED / LIMIT / BREAK).  `log`: the records of
    an episode from its first step on (a fresh DeviceEpisode).  Returns
    [(mpc_problem_t, incumbent)], one per record."""
    ended = MPC_EP_ARRIVED | MPC_EP_LIMIT | MPC_EP_BREAK

    def start():
        return (cfg.start_x, cfg.start_y, cfg.start_phi, 0.0, cfg.target_x, cfg.target_y,
                cfg.start_x, cfg.start_y)

    def criterion0(xt, yt, x0, y0):
        if cfg.incumbent0 != 0.0:
            return cfg.incumbent0
        saved = (mmt.x_t, mmt.y_t, mmt.x_0, mmt.y_0)
        mmt.x_t, mmt.y_t, mmt.x_0, mmt.y_0 = xt, yt, x0, y0
        try:
            return mmt.control_criterion([x0, y0, 0.0])
        finally:
            mmt.x_t, mmt.y_t, mmt.x_0, mmt.y_0 = saved

    x, y, phi, t, xt, yt, x0, y0 = start()
    inc = criterion0(xt, yt, x0, y0)
    out = []
    for rec in log:
        t = t + cfg.delta_t
        out.append((make_problem(x, y, phi, xt, yt, x0, y0, cfg.L, t, t + cfg.delta_t), inc))
        inc = float(sys.maxsize)
        x, y, phi = rec.x, rec.y, rec.phi
        if rec.status & ended:
            x, y, phi, t, xt, yt, x0, y0 = start()
            inc = criterion0(xt, yt, x0, y0)
            continue
        if rec.p == cfg.p_turn_right:
            xt, yt = mmt._turn_target(x, y, phi, cfg.turn_distance, -1)
            x0, y0 = x, y
        if rec.p == cfg.p_turn_left:
            xt, yt = mmt._turn_target(x, y, phi, cfg.turn_distance, +1)
            x0, y0 = x, y
        if rec.p == cfg.p_new_target:
            xt, yt, x0, y0 = cfg.event_target_x, cfg.event_target_y, x, y
    return out


class DeviceEpisode:
    """The same episode with its state in HBM (mpc_episode_* C ABI): a step
    is enqueued without any host synchronisation, so the host only launches
    and the GPU runs steps back to back.  `read_log()` syncs and decodes the
    per-step records (and raises ChainError if a device wait timed out).

    Capturing chained / exchange steps into a hipGraph: end the captured
    sequence with `flush()` inside the capture.  A replay repeats the captured
    launches' epochs; the flush's update clears the published constants' tags,
    without it the next replay's launch with the last epoch could accept the
    previous replay's constants (include/mpc_rollout.h)."""

    def __init__(self, engine, n_cand_total, n_steps, rank=0, world=1, seed=20261015,
                 integrator="rect", group=None, start=(0.0, 0.0, 0.0, 0.0, 0.0), target=(2, 3),
                 log_capacity=4096, split=True, exchange=None, chain=False, L=None,
                 generate=False, max_steps=0, incumbent0=0.0, enumerate=False, overlap=False,
                 p2p=False, mailbox_uncached=True):
        self.eng = engine
        self.lib = native.lib()
        self.n_total = int(n_cand_total)
        self.n_steps = int(n_steps)
        self.rank, self.world, self.group = rank, world, group
        self.lo, self.hi = shard_range(self.n_total, rank, world)
        self.n_local = self.hi - self.lo
        self.integrator = integrator
        self.cfg = reference_episode_config(start, target, seed, max_steps=max_steps,
                                            incumbent0=incumbent0, enumerate=enumerate)
        if L is not None:                 # wheelbase other than config.py's (tests: L not 2^k)
            self.cfg.L = float(L)
        dev = engine.device
        self.state = torch.zeros(self.lib.mpc_episode_state_bytes(), dtype=torch.uint8,
                                 device=dev)
        self.v_sc = torch.empty((self.n_steps, self.n_local), dtype=torch.float64, device=dev)
        self.b_sc = torch.empty_like(self.v_sc)
        self.local = torch.zeros(RESULT_BYTES, dtype=torch.uint8, device=dev)
        self.winner = torch.zeros(RESULT_BYTES, dtype=torch.uint8, device=dev)
        self.log_capacity = int(log_capacity)
        self.log = torch.zeros(self.log_capacity * LOG_BYTES, dtype=torch.uint8, device=dev)
        # zeroed: an exchange step's tagged block records must never find an
        # old allocation's bytes carrying a tag (mpc_episode.h store_tagged_rec)
        self.ws = torch.zeros(self.lib.mpc_workspace_bytes(self.n_local, self.n_steps),
                              dtype=torch.uint8, device=dev)
        from .abi import INTEGRATORS
        self._integ = INTEGRATORS[integrator]
        self.cur = (self.v_sc, self.b_sc)
        self.split = bool(split)
        # exchange: the multi-GPU step structure (finalize -> all_gather ->
        # advance).  Always on for world > 1; forcing it on one rank rehearses
        # the RCCL exchange (and its HIP-graph capture) on a single GPU.
        self.exchange = world > 1 if exchange is None else bool(exchange)
        if world > 1 and not self.exchange:
            raise ValueError("world > 1 needs the exchange step")
        # chain: each step's launch also completes the previous step
        # (mpc_episode_chain_step; caller-resident controls, aligned path);
        # flush() completes the last one.
        self.chain = bool(chain)
        self._ws = [self.ws, torch.zeros_like(self.ws)] if self.chain else [self.ws]
        # exchange + chain: this rank's best candidate of the step (the
        # all_gather payload of mpc_episode_exchange_step)
        self.cand = torch.zeros(CANDIDATE_BYTES, dtype=torch.uint8, device=dev)
        # overlap (exchange + chain): the all_gather of step k runs on a side
        # stream beside launch k+1, whose block 0 waits for its device-side
        # mark (mpc_episode_exchange_step2 / _mark) — see include/mpc_rollout.h
        self.overlap = bool(overlap)
        if self.overlap and not (self.exchange and self.chain):
            raise ValueError("overlap: the chained exchange step only (exchange=True, chain=True)")
        if self.overlap and self.world > 32:
            raise ValueError("overlap: at most 32 ranks (gathered candidates staged in LDS)")
        self._gathered = torch.zeros(self.world * CANDIDATE_BYTES, dtype=torch.uint8, device=dev)
        self._comm = torch.cuda.Stream(device=dev) if self.overlap else None
        # p2p (exchange + chain): no collective — each launch's block 0 stores
        # its rank's candidate into every rank's mailbox over xGMI and the next
        # launch's block 0 waits for the world candidates in its own
        # (mpc_episode_p2p_step); see _p2p_setup
        self.p2p = bool(p2p)
        if self.p2p and (self.overlap or not (self.exchange and self.chain)):
            raise ValueError("p2p: the chained exchange step (exchange=True, chain=True), "
                             "not overlapped")
        self._mailbox, self._opened = None, []
        self.p2p_status = None
        if self.p2p:
            self._p2p_setup(dev, bool(mailbox_uncached))
        self._pend_epoch = 0
        # generate: steps without caller controls draw their candidates inside
        # the rollout (mpc_episode_generate_step) instead of sampling them into
        # v_sc / b_sc first — the same candidates, never written to HBM
        self.generate = bool(generate)
        if self.generate and self.exchange:
            raise ValueError("generated controls: one GPU (no exchange step)")
        self._gen_ws = None
        self._pending = None
        self._epoch = 0
        self._checked = {}
        self.steps_enqueued = 0
        self.reset(_fresh_mailbox=True)

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def _p2p_setup(self, dev, uncached):
        """This rank's mailbox, the ranks' IPC handles exchanged once over the
        process group, the peers' mailboxes opened and written into this
        mailbox's header, then a self-test of the mailboxes (mpc_mailbox_ping)
        on every rank.  If any rank fails any of it, every rank falls back to
        the all_gather exchange (self.p2p = False; the reason in
        self.p2p_status)."""
        L = self.lib
        if self.world > 32:
            raise ValueError("p2p: at most 32 ranks")
        self.p2p_status = "mailbox peer stores"
        ok = 1
        h = (ctypes.c_uint8 * IPC_HANDLE_BYTES)()
        try:
            mb = ctypes.c_void_p()
            with torch.cuda.device(dev):
                native.check(L.mpc_mailbox_alloc(self.world, int(uncached), ctypes.byref(mb)),
                             "mpc_mailbox_alloc")
            self._mailbox = mb.value
            if self.world > 1:
                native.check(L.mpc_ipc_handle(ctypes.c_void_p(self._mailbox), h),
                             "mpc_ipc_handle")
        except RuntimeError as e:
            ok, self.p2p_status = 0, f"fell back to all_gather: {e}"
        if self._all_ok(ok, dev):
            try:
                ptrs = [0] * self.world
                ptrs[self.rank] = self._mailbox
                if self.world > 1:
                    local = torch.tensor(bytearray(h), dtype=torch.uint8, device=dev)
                    handles = gather_bytes(local, self.group).cpu().numpy().reshape(self.world, -1)
                    for r in range(self.world):
                        if r == self.rank:
                            continue
                        p = ctypes.c_void_p()
                        hr = (ctypes.c_uint8 * IPC_HANDLE_BYTES).from_buffer_copy(
                            handles[r].tobytes())
                        with torch.cuda.device(dev):   # mapped for this rank's GPU
                            native.check(L.mpc_ipc_open(hr, ctypes.byref(p)), "mpc_ipc_open")
                        self._opened.append(p.value)
                        ptrs[r] = p.value
                arr = (ctypes.c_void_p * self.world)(*ptrs)
                with torch.cuda.device(dev):
                    native.check(L.mpc_mailbox_set_peers(ctypes.c_void_p(self._mailbox),
                                                         self.rank, self.world, arr),
                                 "mpc_mailbox_set_peers")
            except RuntimeError as e:
                ok, self.p2p_status = 0, f"fell back to all_gather: {e}"
        else:
            ok = 0
        if self._all_ok(ok, dev):
            # every rank's header is written (the all_ok above is a barrier)
            flag = torch.zeros(1, dtype=torch.int32, device=dev)
            with torch.cuda.device(dev):
                native.check(L.mpc_mailbox_ping(ctypes.c_void_p(self._mailbox), 0x5A17,
                                                flag.data_ptr(), self._stream()),
                             "mpc_mailbox_ping")
            ok = int(flag.item())
            if not ok:
                self.p2p_status = "fell back to all_gather: the mailbox self-test timed out"
            ok = self._all_ok(ok, dev)
        else:
            ok = 0
        if not ok:
            if self.p2p_status == "mailbox peer stores":
                self.p2p_status = "fell back to all_gather: a peer's mailbox setup failed"
            self.close()
            self.p2p = False
        self._prev_epoch = 0

    def _all_ok(self, ok, dev):
        """min over the ranks of a 0/1 flag (a collective: every rank calls it)."""
        if self.world == 1:
            return int(ok)
        import torch.distributed as dist
        on_dev = dist.get_backend(self.group) == "nccl"
        t = torch.tensor([int(ok)], dtype=torch.int32, device=dev if on_dev else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.group)
        return int(t.item())

    def close(self):
        """Release the P2P mailbox and the peers' mappings, and let the
        overlapped form's side stream drain (idempotent).  Call it before the
        process group is destroyed: no collective or peer store of this
        episode may still be in flight when the process exits."""
        L = self.lib
        if self._comm is not None:
            self._comm.synchronize()
            torch.cuda.current_stream().synchronize()
        for p in self._opened:
            L.mpc_ipc_close(ctypes.c_void_p(p))
        self._opened = []
        if self._mailbox:
            torch.cuda.synchronize()
            L.mpc_mailbox_free(ctypes.c_void_p(self._mailbox))
            self._mailbox = None

    def reset(self, _fresh_mailbox=False):
        """Restart the episode from cfg.  P2P form: also zeroes this rank's
        mailbox slots (mpc_mailbox_clear), so that no step replayed with an
        epoch of the previous run (a graph captured before the reset) reads a
        stale candidate as fresh; with world > 1 that makes reset() a
        collective — every rank calls it, and none posts into a peer's
        mailbox before every rank has cleared its own.  (A new mailbox is
        zeroed by mpc_mailbox_alloc.)"""
        native.check(self.lib.mpc_episode_reset(ctypes.byref(self.cfg), self.state.data_ptr(),
                                                self._stream()), "mpc_episode_reset")
        self.steps_enqueued = 0
        self._pending = None
        if self.p2p and self._mailbox and not _fresh_mailbox:
            native.check(self.lib.mpc_mailbox_clear(ctypes.c_void_p(self._mailbox), self.world,
                                                    self._stream()), "mpc_mailbox_clear")
            if self.world > 1:
                torch.cuda.current_stream().synchronize()
                self._all_ok(1, self.state.device)      # every rank cleared

    @staticmethod
    def _is_tiled(controls):
        return isinstance(controls, torch.Tensor)

    def _ptrs(self, controls):
        """(v pointer, beta pointer, integrator id) of a checked control batch:
        SoA (v, beta) or a tiled tensor (MPC_LAYOUT_TILED: beta = v + 512)."""
        from .abi import MPC_LAYOUT_TILED, MPC_TILE
        if self._is_tiled(controls):
            p = controls.data_ptr()
            return p, p + 8 * MPC_TILE, self._integ | MPC_LAYOUT_TILED
        v, b = controls
        return v.data_ptr(), b.data_ptr(), self._integ

    def _seen(self, key, *tensors):
        """Was this very batch (same tensor objects) checked before?  The cache
        holds weak references only: a caller's per-step batches are not kept
        alive by it (and a new tensor reusing a freed one's id and memory is
        not mistaken for it)."""
        refs = self._checked.get(key)
        return refs is not None and all(r() is t for r, t in zip(refs, tensors))

    def _remember(self, key, *tensors):
        if len(self._checked) >= 4096:
            self._checked = {k: r for k, r in self._checked.items()
                             if all(x() is not None for x in r)}
            if len(self._checked) >= 4096:
                self._checked.clear()
        self._checked[key] = tuple(weakref.ref(t) for t in tensors)

    def _check_controls(self, controls):
        if self._is_tiled(controls):
            return self._check_tiled(controls)
        v, b = controls
        key = (id(v), id(b), v.data_ptr(), b.data_ptr())
        if self._seen(key, v, b):        # a resident batch seen before: checked once
            return v, b
        if (tuple(v.shape) != (self.n_steps, self.n_local) or v.shape != b.shape
                or v.dtype != torch.float64 or b.dtype != torch.float64
                or not v.is_contiguous() or not b.is_contiguous()
                or v.device != self.v_sc.device or b.device != self.v_sc.device):
            raise ValueError("controls must be contiguous float64 [n_steps, n_local] "
                             "tensors on the episode's device")
        self._remember(key, v, b)
        return v, b

    def _check_tiled(self, t):
        from .abi import MPC_TILE
        key = (id(t), t.data_ptr())
        if self._seen(key, t):
            return t
        if (tuple(t.shape) != (-(-self.n_local // MPC_TILE), self.n_steps, 2, MPC_TILE)
                or t.dtype != torch.float64 or not t.is_contiguous()
                or t.device != self.v_sc.device or t.data_ptr() % 16):
            raise ValueError("tiled controls must be a contiguous 16-B aligned float64 "
                             "[ceil(n_local / 512), n_steps, 2, 512] tensor on the episode's "
                             "device (Expansion.sample_controls_tiled)")
        self._remember(key, t)
        return t

    def _chain_step(self, controls, events=None):
        """One chained launch: this step's rollout + the previous step's
        completion (one GPU: finalize + update; multi-GPU: selection over the
        gathered winners + update), then on multi-GPU this step's local
        finalize and the all_gather."""
        L, st = self.lib, self._stream()
        ctl = self._check_controls(controls)
        tiled = self._is_tiled(ctl)
        if tiled and self.exchange and not self.p2p:
            raise ValueError("tiled controls: the one-GPU and P2P chained steps only")
        self.cur = ctl
        vp, bp, integ = self._ptrs(ctl)
        ws, ws_prev = self._ws[0], self._ws[1]
        pend = self._pending
        pv = pb = None
        if not self.exchange or self.p2p:   # (the all_gather forms pend the gathered bytes)
            if pend is not None and self._is_tiled(pend) != tiled:
                raise ValueError("a chained episode keeps one control layout until its flush")
            if pend is not None:
                pv, pb = self._ptrs(pend)[:2]
        if events:
            events[0].record()
        if not self.exchange:
            native.check(L.mpc_episode_chain_step(
                ctypes.byref(self.cfg), self.state.data_ptr(), 1, self._next_epoch(),
                vp, bp,
                self.n_local, self.n_steps, self.lo, integ, ws.data_ptr(),
                ws_prev.data_ptr(), ws.numel(), pv, pb, self.local.data_ptr(), None, 0,
                self.log.data_ptr(), self.log_capacity, st), "mpc_episode_chain_step")
            self._pending = ctl
        elif self.p2p:
            # one launch: rollout of step k; its block 0 completes step k-1 —
            # this rank's candidate posted to every mailbox over xGMI, the
            # world's awaited, selection + update (no collective, no host step)
            epoch = self._next_epoch()
            native.check(L.mpc_episode_p2p_step(
                ctypes.byref(self.cfg), self.state.data_ptr(), epoch,
                self._prev_epoch if pend is not None else 0, vp, bp,
                self.n_local, self.n_steps, self.lo, integ, ws.data_ptr(),
                ws_prev.data_ptr(), ws.numel(), pv, pb, ctypes.c_void_p(self._mailbox),
                self.world, self.winner.data_ptr(), self.log.data_ptr(), self.log_capacity, st),
                "mpc_episode_p2p_step")
            self._pending = ctl
            self._prev_epoch = epoch
        elif not self.overlap:
            # one launch (selection of step k-1 over the gathered candidates +
            # the rollout of step k + this rank's candidate), then ONE
            # all_gather of the 536-B candidates
            native.check(L.mpc_episode_exchange_step(
                ctypes.byref(self.cfg), self.state.data_ptr(), self._next_epoch(),
                vp, bp, self.n_local, self.n_steps, self.lo, self._integ,
                ws.data_ptr(), ws.numel(), pend.data_ptr() if pend is not None else None,
                self.world if pend is not None else 0, self.winner.data_ptr(),
                self.cand.data_ptr(), self.log.data_ptr(), self.log_capacity, st),
                "mpc_episode_exchange_step")
            if events:                   # the launch alone, not the collective after it
                events[1].record()
                events = None
            self._pending = gather_bytes(self.cand, self.group)
        else:
            # the same launch, but the collective of the previous step may
            # still be running beside it: block 0 waits for its mark
            _check_overlap_stream()
            epoch = self._next_epoch()
            native.check(L.mpc_episode_exchange_step2(
                ctypes.byref(self.cfg), self.state.data_ptr(), epoch,
                self._pend_epoch if pend is not None else 0, vp, bp,
                self.n_local, self.n_steps, self.lo, self._integ, ws.data_ptr(), ws.numel(),
                self._gathered.data_ptr() if pend is not None else None,
                self.world if pend is not None else 0, self.winner.data_ptr(),
                self.cand.data_ptr(), self.log.data_ptr(), self.log_capacity, st),
                "mpc_episode_exchange_step2")
            if events:
                events[1].record()
                events = None
            main = torch.cuda.current_stream()
            self._comm.wait_stream(main)          # after this launch (its candidate)
            with torch.cuda.stream(self._comm):
                gather_into(self._gathered, self.cand, self.group)
                native.check(L.mpc_episode_exchange_mark(
                    self.state.data_ptr(), epoch,
                    ctypes.c_void_p(self._comm.cuda_stream)), "mpc_episode_exchange_mark")
            self._pending = self._gathered
            self._pend_epoch = epoch
        if events:
            events[1].record()
        if pend is not None:
            self.steps_enqueued += 1
        self._ws.reverse()

    def run(self, batches):
        """len(batches) COMPLETE MPC steps in one persistent launch per 64
        (mpc_episode_run, csrc/mpc_run.h): step j over batches[j] — each a
        resident SoA (v, beta) pair or a tiled tensor, one layout for the run.
        One GPU, rect+cum, the chained step's controls; the log, the state and
        `local` (the last step's winner) equal those of the same chained steps
        and their flush, bit for bit.  A pending chained step is completed
        first."""
        if self.exchange:
            raise ValueError("the persistent run: one GPU (no exchange step)")
        if self.integrator != "rect+cum" or self.n_local % 2:
            raise ValueError("the persistent run streams rect+cum candidates, n_local even")
        batches = list(batches)
        if not batches:
            return
        self.flush()
        ctls = [self._check_controls(c) for c in batches]
        tiled = self._is_tiled(ctls[0])
        if any(self._is_tiled(c) != tiled for c in ctls):
            raise ValueError("one control layout per run")
        if not tiled and any(not self._chainable(c) for c in ctls):
            raise ValueError("SoA controls of a run must be 16-B aligned")
        ptrs = [self._ptrs(c) for c in ctls]
        k = len(ptrs)
        V = (ctypes.c_void_p * k)(*[p[0] for p in ptrs])
        B = (ctypes.c_void_p * k)(*[p[1] for p in ptrs])
        if getattr(self, "_run_ws", None) is None:
            # zeroed once; every run leaves it zeroed (tagged records consumed)
            self._run_ws = torch.zeros(self.lib.mpc_episode_run_workspace_bytes(self.n_local),
                                       dtype=torch.uint8, device=self.state.device)
        # k consecutive nonzero epochs (the published constants' tags)
        if self._epoch + k >= 0xFFFFFFF0:
            self._epoch = 0
        e0 = self._epoch + 1
        self._epoch += k
        native.check(self.lib.mpc_episode_run(
            ctypes.byref(self.cfg), self.state.data_ptr(), e0, V, B, k, self.n_local,
            self.n_steps, self.lo, ptrs[0][2], self._run_ws.data_ptr(), self._run_ws.numel(),
            self.local.data_ptr(), self.log.data_ptr(), self.log_capacity, self._stream()),
            "mpc_episode_run")
        self.cur = ctls[-1]
        self.steps_enqueued += k

    def _next_epoch(self):
        # nonzero, differs from the last and in parity (the P2P mailbox's two
        # slots alternate: 0xFFFFFFFE is followed by 1)
        self._epoch = self._epoch % 0xFFFFFFFE + 1
        return self._epoch

    def flush(self):
        """Complete the step a chained launch left pending (no-op otherwise)."""
        pend, self._pending = self._pending, None
        if pend is None:
            return
        L, st = self.lib, self._stream()
        if not self.exchange:
            vp, bp, integ = self._ptrs(pend)
            native.check(L.mpc_episode_finalize(
                self.state.data_ptr(), vp, bp, self.n_local, self.n_steps,
                self.lo, integ, self._ws[1].data_ptr(), self._ws[1].numel(),
                self.local.data_ptr(), ctypes.byref(self.cfg), self.log.data_ptr(),
                self.log_capacity, st), "mpc_episode_finalize")
        elif self.p2p:
            vp, bp, integ = self._ptrs(pend)
            native.check(L.mpc_episode_p2p_flush(
                ctypes.byref(self.cfg), self.state.data_ptr(), self._prev_epoch, vp,
                bp, self.n_local, self.n_steps, self.lo, integ,
                self._ws[1].data_ptr(), self._ws[1].numel(), ctypes.c_void_p(self._mailbox),
                self.world, self.winner.data_ptr(), self.log.data_ptr(), self.log_capacity, st),
                "mpc_episode_p2p_flush")
        else:
            if self.overlap:                      # the last collective, then its step
                torch.cuda.current_stream().wait_stream(self._comm)
            native.check(L.mpc_episode_exchange_flush(
                ctypes.byref(self.cfg), self.state.data_ptr(), self._integ, pend.data_ptr(),
                self.world, self.winner.data_ptr(), self.log.data_ptr(), self.log_capacity, st),
                "mpc_episode_exchange_flush")
        self.steps_enqueued += 1

    def chain_error(self, local=False):
        """EpisodeState::chain_error — with world > 1 the MAX over the ranks (a
        collective: every rank calls it), since a rank whose wait timed out
        posted nothing, so its peers' steps diverge from the true arg-min
        while their own code stays 0.  local=True: this rank's code only."""
        e = ctypes.c_int32(0)
        native.check(self.lib.mpc_episode_chain_error(self.state.data_ptr(), ctypes.byref(e),
                                                      self._stream()), "mpc_episode_chain_error")
        err = int(e.value)
        if self.world > 1 and not local:
            import torch.distributed as dist
            on_dev = dist.get_backend(self.group) == "nccl"
            t = torch.tensor([err], dtype=torch.int32,
                             device=self.state.device if on_dev else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
            err = int(t.item())
        return err

    def expand(self, events=None, controls=None):
        """Grid + sampler + rollout + finalize for this rank's shard.
        controls: optional caller-resident (v_sc, beta_sc) fp64 [n_steps,
        n_local] for this step — the rollout streams them instead of the
        sampler's (the candidate set is the caller's input).
        events: optional (start, stop) torch.cuda.Event pair recorded around
        the rollout (+ selection) launch."""
        st = self._stream()
        L = self.lib
        self.flush()
        if controls is None and self.generate:
            if self.exchange:
                raise ValueError("generated controls: one GPU (no exchange step)")
            if self._gen_ws is None:
                self._gen_ws = torch.empty(self.lib.mpc_episode_generate_workspace_bytes(
                    self.n_local, self.n_steps), dtype=torch.uint8, device=self.state.device)
            if events:
                events[0].record()
            native.check(L.mpc_episode_generate_step(
                ctypes.byref(self.cfg), self.state.data_ptr(), self.n_local, self.n_steps,
                self.lo, self._integ, self._gen_ws.data_ptr(), self._gen_ws.numel(),
                self.local.data_ptr(), self.log.data_ptr(), self.log_capacity, st),
                "mpc_episode_generate_step")
            if events:
                events[1].record()
            self.steps_enqueued += 1
            return
        if controls is None:
            native.check(L.mpc_episode_sample(ctypes.byref(self.cfg), self.state.data_ptr(),
                                              self.v_sc.data_ptr(), self.b_sc.data_ptr(),
                                              self.n_local, self.n_steps, self.lo, st),
                         "mpc_episode_sample")
            self.cur = (self.v_sc, self.b_sc)
        else:
            self.cur = self._check_controls(controls)
        one_gpu = not self.exchange  # one GPU: the step's launch also advances the episode
        args = (self.state.data_ptr(), self.cur[0].data_ptr(), self.cur[1].data_ptr(),
                self.n_local, self.n_steps, self.lo, self._integ, self.ws.data_ptr(),
                self.ws.numel(), self.local.data_ptr(),
                ctypes.byref(self.cfg) if one_gpu else None,
                self.log.data_ptr() if one_gpu else None, self.log_capacity if one_gpu else 0, st)
        if events:
            events[0].record()
        if self.split and not events:
            # streaming kernel, then the selection kernel: two launches in one
            # host call (the faster form on MI355X: 44.8 vs 47.5 us per
            # config-C step than the one-launch form below)
            native.check(L.mpc_episode_step(*args), "mpc_episode_step")
        elif self.split:
            self.partials(st)
            native.check(L.mpc_episode_finalize(*args), "mpc_episode_finalize")
        else:
            # one launch: the last block to finish runs the selection
            native.check(L.mpc_episode_rollout(*args), "mpc_episode_rollout")
        if events:
            events[1].record()
        if one_gpu:
            self.steps_enqueued += 1

    def partials(self, st=None):
        """The streaming rollout/arg-min kernel alone on the current controls
        (writes only the workspace block records; the episode is unchanged)."""
        self.flush()
        if self._is_tiled(self.cur):
            raise ValueError("the streaming kernel alone reads SoA controls")
        v, b = self.cur
        native.check(self.lib.mpc_episode_partials(
            self.state.data_ptr(), v.data_ptr(), b.data_ptr(), self.n_local,
            self.n_steps, self._integ, self.ws.data_ptr(), self.ws.numel(),
            st if st is not None else self._stream()), "mpc_episode_partials")

    def advance(self):
        """Multi-GPU: all_gather of the per-rank winners (RCCL) + selection +
        episode update in one launch; no host synchronisation.  (On one GPU
        the update already ran inside finalize.)"""
        if not self.exchange:
            return
        gathered = gather_results(self.local, self.group)
        native.check(self.lib.mpc_episode_advance(
            ctypes.byref(self.cfg), self.state.data_ptr(), gathered.data_ptr(), self.world,
            self.log.data_ptr(), self.log_capacity, self._stream()), "mpc_episode_advance")
        self.steps_enqueued += 1

    def step(self, events=None, controls=None):
        """One MPC step.  controls: this step's resident candidates — SoA
        (v_sc, beta_sc) [n_steps, n_local] or, for the chained steps (one GPU or
        P2P), a tiled tensor (Expansion.sample_controls_tiled); None: the
        device sampler draws them."""
        if self.chain and controls is not None and self._chainable(controls):
            self._chain_step(controls, events)
            return
        if controls is not None and self._is_tiled(controls):
            raise ValueError("tiled controls: chained rect+cum steps only (chain=True)")
        self.expand(events, controls)
        self.advance()

    def _chainable(self, controls):
        if self._is_tiled(controls):
            return self.integrator == "rect+cum" and self.n_local % 2 == 0
        v, b = controls
        return (self.integrator == "rect+cum" and self.n_local % 2 == 0
                and v.data_ptr() % 16 == 0 and b.data_ptr() % 16 == 0)

    def read_log(self):
        """Complete any pending step, sync, and decode the per-step records.
        Raises ChainError if a chained / exchange step's bounded device wait
        timed out on ANY rank (chain_error(), reduced over the ranks): such a
        step ran on speculated constants or dropped a rank's candidate, so
        the log records must not be trusted.  With world > 1 every rank must
        call it (the reduction is a collective)."""
        self.flush()
        torch.cuda.current_stream().synchronize()
        err = self.chain_error()
        if err:
            raise ChainError(err)
        # the log is complete: one copy into pinned host memory (a staged copy
        # to pageable memory left an async-copy completion callback undelivered
        # at process exit under rocprofv3's memory-copy tracing,
        # profiles/r06/overlap_exit/)
        if getattr(self, "_log_host", None) is None:
            self._log_host = torch.empty(self.log.numel(), dtype=torch.uint8).pin_memory()
        self._log_host.copy_(self.log, non_blocking=True)
        torch.cuda.current_stream().synchronize()
        raw = self._log_host.numpy().tobytes()
        n = min(self.steps_enqueued, self.log_capacity)
        recs = [MpcEpisodeLog.from_buffer_copy(raw[i * LOG_BYTES:(i + 1) * LOG_BYTES])
                for i in range(self.log_capacity)]
        # a written record has episode >= 1 (slots never written are zero)
        recs = [r for r in recs if r.episode >= 1 and r.step < self.steps_enqueued]
        recs.sort(key=lambda r: r.step)
        return recs[-n:]


def percentile(xs, q):
    if not xs:
        return math.nan
    s = sorted(xs)
    i = min(len(s) - 1, max(0, int(round(q / 100.0 * (len(s) - 1)))))
    return s[i]


# numpy view of mpc_episode_log_t (include/mpc_rollout.h), 80 bytes
_LOG_DTYPE = [("step", "<i8"), ("index", "<i8"), ("p", "<i4"), ("episode", "<i4"),
              ("found", "<i4"), ("status", "<i4"), ("cost", "<f8"), ("x", "<f8"), ("y", "<f8"),
              ("phi", "<f8"), ("v", "<f8"), ("beta", "<f8")]


class DeviceEpisodes:
    """R robots' MPC episodes in HBM (mpc_episodes_*, csrc/mpc_episodes.h):
    one block per robot runs its episode's MPC steps back to back — the grid
    around its control, the reference's enumeration of the step's |V| x |B|
    constant sequences, the N-step rollout, the strict-< first minimum, the
    winner's layer states and the episode update — so `run(k)` is ONE launch
    for up to k MPC steps of every robot, with no host round trip and no
    lockstep.  cfgs: one MpcEpisodeConfig per robot (start, target and rules:
    `tree_episode_config` for run_math_model.py's loop, the reference_episode_
    config of math_mpc for the operator scenario)."""

    def __init__(self, engine, cfgs, n_steps=3, integrator="qk21", log_capacity=1024):
        from .abi import INTEGRATORS, PROGRESS_BYTES
        self.eng = engine
        self.lib = native.lib()
        self.cfgs = list(cfgs)
        self.R = len(self.cfgs)
        self.n_steps = int(n_steps)
        self.integrator = integrator
        self._integ = INTEGRATORS[integrator]
        dev = engine.device
        self.state = torch.zeros(self.lib.mpc_episodes_state_bytes(self.R), dtype=torch.uint8,
                                 device=dev)
        self.log_capacity = int(log_capacity)
        self.log = torch.zeros(self.R * self.log_capacity * LOG_BYTES, dtype=torch.uint8,
                               device=dev)
        self.progress = torch.zeros(self.R * PROGRESS_BYTES, dtype=torch.uint8, device=dev)
        self.reset()

    def reset(self):
        arr = (MpcEpisodeConfig * self.R)(*self.cfgs)
        native.check(self.lib.mpc_episodes_reset(ctypes.byref(arr), self.R, self.state.data_ptr(),
                                                 _stream()), "mpc_episodes_reset")
        self.progress.zero_()

    def run(self, max_calls):
        """Enqueue up to max_calls MPC steps of every still-running robot."""
        native.check(self.lib.mpc_episodes_run(
            self.state.data_ptr(), self.R, self.n_steps, self._integ, int(max_calls),
            self.log.data_ptr(), self.log_capacity, self.progress.data_ptr(), _stream()),
            "mpc_episodes_run")

    def read_progress(self):
        """(calls, stop, candidates) per robot (numpy arrays; syncs)."""
        import numpy as np
        raw = self.progress.cpu().numpy()
        p = np.frombuffer(raw.tobytes(), dtype=[("calls", "<i4"), ("stop", "<i4"),
                                                ("candidates", "<i8")])
        return p["calls"].copy(), p["stop"].copy(), p["candidates"].copy()

    def read_logs(self, first_step=None):
        """Per robot, its log records (numpy structured array, mpc_episode_log_t
        fields) of steps [first, calls): first = first_step[r] if given, else
        everything still in the ring (the last log_capacity steps)."""
        import numpy as np
        calls, _, _ = self.read_progress()
        raw = np.frombuffer(self.log.cpu().numpy().tobytes(), dtype=_LOG_DTYPE)
        raw = raw.reshape(self.R, self.log_capacity)
        out = []
        for r in range(self.R):
            n = int(calls[r])
            lo = max(0, n - self.log_capacity)
            if first_step is not None:
                lo = max(lo, int(first_step[r]))
            out.append(raw[r, [s % self.log_capacity for s in range(lo, n)]])
        return out


class DeviceFtEpisodes:
    """R robots' run_math_model.py episodes with the script's own full-tree MPC
    step, in HBM (mpc_fulltree_episodes_*, csrc/mpc_ftepisodes.h): `run(k)`
    enqueues up to k calls of every robot with no host step in between — per
    call the robots still running are compacted and every one's S1^3 leaves
    are spread over the whole GPU (the load-balanced lockstep form).  cfgs:
    MpcFulltreeEpisodeConfig per robot; v_grid / beta_grid: the script's grids
    as device tensors."""

    def __init__(self, engine, cfgs, v_grid, beta_grid, L, delta_t, eps, integrator="qk21",
                 log_capacity=256):
        from .abi import INTEGRATORS, MpcFulltreeEpisodeConfig, PROGRESS_BYTES
        self.lib = native.lib()
        self.cfgs = (MpcFulltreeEpisodeConfig * len(cfgs))(*cfgs)
        self.R = len(cfgs)
        self.vg, self.bg = v_grid, beta_grid
        self.L, self.delta_t, self.eps = float(L), float(delta_t), float(eps)
        self._integ = INTEGRATORS[integrator]
        dev = engine.device
        self.state = torch.zeros(self.lib.mpc_fulltree_episodes_state_bytes(self.R),
                                 dtype=torch.uint8, device=dev)
        self.log_capacity = int(log_capacity)
        self.log = torch.zeros(self.R * self.log_capacity * LOG_BYTES, dtype=torch.uint8,
                               device=dev)
        self.progress = torch.zeros(self.R * PROGRESS_BYTES, dtype=torch.uint8, device=dev)
        self.reset()

    def reset(self):
        native.check(self.lib.mpc_fulltree_episodes_reset(ctypes.byref(self.cfgs), self.R,
                                                          self.state.data_ptr(), _stream()),
                     "mpc_fulltree_episodes_reset")
        self.progress.zero_()

    def run(self, max_calls):
        """Enqueue up to max_calls MPC calls of every still-running robot
        (three launches per call, each bounded by one call's S1^3 leaves per
        robot spread over the GPU: no launch approaches the compute-lockup
        timeout whatever S1 and max_calls are)."""
        native.check(self.lib.mpc_fulltree_episodes_run(
            self.state.data_ptr(), self.R, self.vg.data_ptr(), self.vg.numel(),
            self.bg.data_ptr(), self.bg.numel(), self.L, self.delta_t, self.eps, self._integ,
            int(max_calls), self.log.data_ptr(), self.log_capacity, self.progress.data_ptr(),
            _stream()), "mpc_fulltree_episodes_run")

    read_progress = DeviceEpisodes.read_progress   # (calls, stop, leaves) per robot
    read_logs = DeviceEpisodes.read_logs


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


_CU_RESERVED = set()   # handles of the streams cu_reserved_stream() made


def _check_overlap_stream():
    """An overlapped exchange launch must leave CUs to the collective that runs
    beside it: a launch larger than one resident round (config C: 1954 blocks,
    1536 resident) fills every CU with blocks that wait, at the end of their
    tile, for block 0 — which waits for the collective.  Eager launches must
    therefore go to a cu_reserved_stream().  Eager only: a replayed hipGraph
    runs its parallel branches on runtime streams that carry no CU mask
    (measured: the 1M-candidate graph's launches filled every CU and block 0
    timed out, chain error 4)."""
    if torch.cuda.is_current_stream_capturing():
        raise ValueError("overlapped exchange: eager launches only (a replayed graph's branches "
                         "lose the launch stream's CU mask)")
    if torch.cuda.current_stream().cuda_stream in _CU_RESERVED:
        return
    raise ValueError("overlapped exchange: launch on a cu_reserved_stream() so the collective "
                     "beside each launch finds free CUs")


def cu_reserved_stream(device, reserved_per_xcd=1):
    """A torch stream whose kernels (and hipGraphs replayed on it) leave
    `reserved_per_xcd` CUs of every XCD free (mpc_stream_create_cu_reserved):
    the launch stream of the overlapped exchange (DeviceEpisode(overlap=True)),
    so that the collective running beside a chained launch always finds CUs.
    Lives until the process exits: an atexit hook synchronises the device and
    destroys it (before the HIP runtime's own teardown, which otherwise finds
    a stream it did not create still registered)."""
    lib = native.lib()
    p = ctypes.c_void_p()
    with torch.cuda.device(device):
        native.check(lib.mpc_stream_create_cu_reserved(int(reserved_per_xcd), ctypes.byref(p)),
                     "mpc_stream_create_cu_reserved")
    if reserved_per_xcd > 0:
        _CU_RESERVED.add(p.value)
    if not _CREATED:
        import atexit
        atexit.register(_destroy_streams)
    _CREATED.append((p.value, torch.device(device)))
    return torch.cuda.ExternalStream(p.value, device=device)


def cu_share_stream(device, part, parts):
    """A torch stream on the part-th of `parts` disjoint CU sets of the device
    (mpc_stream_create_cu_share): the launch stream of each of several ranks
    that rehearse a multi-GPU run on ONE GPU.  A chained exchange launch
    larger than one resident round fills every CU with tile blocks waiting for
    block 0, which waits for the peers — whose launches then find no CU.  On
    disjoint sets every rank keeps CUs for its block 0.  Destroyed at exit."""
    lib = native.lib()
    p = ctypes.c_void_p()
    with torch.cuda.device(device):
        native.check(lib.mpc_stream_create_cu_share(int(part), int(parts), ctypes.byref(p)),
                     "mpc_stream_create_cu_share")
    if not _CREATED:
        import atexit
        atexit.register(_destroy_streams)
    _CREATED.append((p.value, torch.device(device)))
    return torch.cuda.ExternalStream(p.value, device=device)


_CREATED = []   # (handle, device) of every stream these helpers made


def _destroy_streams():
    """atexit: drain and destroy the streams cu_reserved_stream() made."""
    lib = native.lib()
    while _CREATED:
        h, dev = _CREATED.pop()
        try:
            with torch.cuda.device(dev):
                torch.cuda.synchronize()
                torch.cuda.set_stream(torch.cuda.default_stream(dev))
            lib.mpc_stream_destroy(ctypes.c_void_p(h))
        except Exception:   # the runtime is already gone: nothing left to release
            pass
        _CU_RESERVED.discard(h)


def tree_episode_config(start, max_calls=None):
    """mpc_episode_config_t of one run_math_model.py episode (:231-280) whose
    MPC step is math_model_tree.py's tree expansion (SURVEY Fact 2): start =
    (x_0, y_0, phi_0, x_t, y_t) as draw_starts() draws them, v = beta = 0
    (:233-234); the reference's grid constants and enumeration; the first
    incumbent from the start with the episode's target (:252); no operator
    events; the script's stuck rule (the second non-moving step stops it,
    :266-272); max_calls (None: none) as the step limit."""
    x0, y0, phi0, xt, yt = start
    c = reference_episode_config(start=(float(x0), float(y0), float(phi0), 0.0, 0.0),
                                 target=(float(xt), float(yt)), max_steps=max_calls or 0,
                                 enumerate=True)
    c.p_turn_right = c.p_turn_left = c.p_new_target = 0
    c.stop_rule = 1
    return c
