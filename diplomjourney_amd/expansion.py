"""Device-side MPC candidate expansion: a thin PyTorch-ROCm host over the C ABI.

`Expansion` owns, per device, the workspace and result buffers the C ABI
borrows.  Candidate control sequences live in HBM as fp64 SoA tensors
`[n_steps, n_cand]` (include/mpc_rollout.h).  Every call is asynchronous on
the current torch stream; `fetch()` is the single device->host read per MPC
step that the reference's host loop needs (math_model_tree.py:550).
"""
import ctypes
import math

import torch

from . import native
from .abi import (INTEGRATORS, MPC_MAX_STEPS, RESULT_BYTES, PROBLEM_BYTES, MpcProblem,
                  MpcResult, result_from_bytes)


def _stream_ptr():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _integ(name_or_id):
    if isinstance(name_or_id, str):
        return INTEGRATORS[name_or_id]
    return int(name_or_id)


def _check_soa(t, name, n_steps=None, n_cand=None):
    if not (isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == torch.float64):
        raise TypeError(f"{name} must be a CUDA(HIP) float64 tensor")
    if t.dim() != 2 or not t.is_contiguous():
        raise ValueError(f"{name} must be a contiguous [n_steps, n_cand] tensor")
    if n_steps is not None and t.shape[0] != n_steps:
        raise ValueError(f"{name} has {t.shape[0]} steps, expected {n_steps}")
    if n_cand is not None and t.shape[1] != n_cand:
        raise ValueError(f"{name} has {t.shape[1]} candidates, expected {n_cand}")


class Expansion:
    """Rollout + cost + arg-min engine bound to one HIP device."""

    def __init__(self, device=None):
        self.device = torch.device(device if device is not None else "cuda")
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.lib = native.lib()
        self._ws = torch.empty(0, dtype=torch.uint8, device=self.device)
        self.result = torch.zeros(RESULT_BYTES, dtype=torch.uint8, device=self.device)
        self._host = torch.zeros(RESULT_BYTES, dtype=torch.uint8).pin_memory()

    # -- workspace -----------------------------------------------------------
    def _workspace(self, nbytes):
        if self._ws.numel() < nbytes:
            self._ws = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=self.device)
        return self._ws

    # -- single problem --------------------------------------------------------
    def rollout_argmin(self, problem: MpcProblem, v_sc, beta_sc, index_base=0,
                       incumbent=math.inf, integrator="qk21", states=None, out=None):
        """Enqueue the expansion of one problem; returns the device result buffer.

        states: optional float64 tensor [n_steps, 3, n_cand] receiving every
        candidate's (x, y, phi) after every step (the CoordinateTree payload).
        """
        _check_soa(v_sc, "v_sc")
        n_steps, n_cand = v_sc.shape
        _check_soa(beta_sc, "beta_sc", n_steps, n_cand)
        if not 1 <= n_steps <= MPC_MAX_STEPS:
            raise ValueError(f"n_steps must be in [1, {MPC_MAX_STEPS}]")
        if states is not None:
            if (states.dtype != torch.float64 or not states.is_cuda or not states.is_contiguous()
                    or tuple(states.shape) != (n_steps, 3, n_cand)):
                raise ValueError("states must be a contiguous float64 [n_steps, 3, n_cand] tensor")
        out = self.result if out is None else out
        ws_bytes = self.lib.mpc_workspace_bytes(n_cand, n_steps)
        ws = self._workspace(ws_bytes)
        st = self.lib.mpc_rollout_argmin(
            ctypes.byref(problem), v_sc.data_ptr(), beta_sc.data_ptr(), n_cand, n_steps,
            int(index_base), float(incumbent), _integ(integrator),
            states.data_ptr() if states is not None else None,
            ws.data_ptr(), ws.numel(), out.data_ptr(), _stream_ptr())
        native.check(st, "mpc_rollout_argmin")
        return out

    def partials(self, problem: MpcProblem, v_sc, beta_sc, integrator="qk21"):
        """Phase 1 only: the streaming rollout kernel (block arg-min records)."""
        n_steps, n_cand = v_sc.shape
        ws = self._workspace(self.lib.mpc_workspace_bytes(n_cand, n_steps))
        st = self.lib.mpc_rollout_partials(ctypes.byref(problem), v_sc.data_ptr(),
                                           beta_sc.data_ptr(), n_cand, n_steps,
                                           _integ(integrator), None, ws.data_ptr(), ws.numel(),
                                           _stream_ptr())
        native.check(st, "mpc_rollout_partials")

    def finalize(self, problem: MpcProblem, v_sc, beta_sc, index_base=0, incumbent=math.inf,
                 integrator="qk21", out=None):
        """Phase 2 only: block records -> winner record (device)."""
        n_steps, n_cand = v_sc.shape
        out = self.result if out is None else out
        ws = self._workspace(self.lib.mpc_workspace_bytes(n_cand, n_steps))
        st = self.lib.mpc_rollout_finalize(ctypes.byref(problem), v_sc.data_ptr(),
                                           beta_sc.data_ptr(), n_cand, n_steps, int(index_base),
                                           float(incumbent), _integ(integrator), 0,
                                           ws.data_ptr(), ws.numel(), out.data_ptr(),
                                           _stream_ptr())
        native.check(st, "mpc_rollout_finalize")
        return out

    def fetch(self, out=None) -> MpcResult:
        """Copy one device result to the host (synchronises the stream)."""
        out = self.result if out is None else out
        self._host.copy_(out, non_blocking=True)
        torch.cuda.current_stream().synchronize()
        return result_from_bytes(self._host.numpy().tobytes())

    # -- robots batch --------------------------------------------------------
    def rollout_argmin_batched(self, problems_dev, v_sc, beta_sc, cand_per_problem,
                               incumbents_dev=None, integrator="qk21", out=None):
        """problems_dev: uint8 CUDA tensor of R*sizeof(mpc_problem_t) bytes
        (see `problems_to_device`); returns the device result array [R] bytes."""
        _check_soa(v_sc, "v_sc")
        n_steps, total = v_sc.shape
        _check_soa(beta_sc, "beta_sc", n_steps, total)
        R = problems_dev.numel() // PROBLEM_BYTES
        if R * cand_per_problem != total:
            raise ValueError("v_sc columns must equal n_problems * cand_per_problem")
        if out is None:
            out = torch.zeros(R * RESULT_BYTES, dtype=torch.uint8, device=self.device)
        ws = self._workspace(self.lib.mpc_batched_workspace_bytes(R, cand_per_problem, n_steps))
        st = self.lib.mpc_rollout_argmin_batched(
            problems_dev.data_ptr(),
            incumbents_dev.data_ptr() if incumbents_dev is not None else None,
            R, v_sc.data_ptr(), beta_sc.data_ptr(), cand_per_problem, n_steps,
            _integ(integrator), ws.data_ptr(), ws.numel(), out.data_ptr(), _stream_ptr())
        native.check(st, "mpc_rollout_argmin_batched")
        return out

    # -- multi-GPU exchange ----------------------------------------------------
    def select_winner(self, gathered, incumbent=math.inf, out=None):
        """gathered: uint8 CUDA tensor of n * sizeof(mpc_result_t) (all_gather output)."""
        n = gathered.numel() // RESULT_BYTES
        out = self.result if out is None else out
        st = self.lib.mpc_select_winner(gathered.data_ptr(), n, float(incumbent),
                                        out.data_ptr(), _stream_ptr())
        native.check(st, "mpc_select_winner")
        return out

    # -- synthetic candidates --------------------------------------------------
    def sample_controls(self, v_grid, beta_grid, n_cand, n_steps, seed, index_base=0,
                        const_prefix=True, v_out=None, beta_out=None, ld=None):
        if v_out is None:
            v_out = torch.empty((n_steps, n_cand), dtype=torch.float64, device=self.device)
            beta_out = torch.empty_like(v_out)
        ld = v_out.shape[1] if ld is None else ld
        st = self.lib.mpc_sample_controls(
            v_grid.data_ptr(), v_grid.numel(), beta_grid.data_ptr(), beta_grid.numel(),
            n_cand, n_steps, int(seed) & 0xFFFFFFFFFFFFFFFF, int(index_base), int(const_prefix),
            v_out.data_ptr(), beta_out.data_ptr(), ld, _stream_ptr())
        native.check(st, "mpc_sample_controls")
        return v_out, beta_out

    def sample_controls_tiled(self, v_grid, beta_grid, n_cand, n_steps, seed, index_base=0,
                              const_prefix=True):
        """The same candidates as sample_controls in the TILED layout
        (MPC_LAYOUT_TILED): a tensor [tiles, n_steps, 2, MPC_TILE] (v then
        beta per tile and step); tiled_to_soa() gives the SoA view's values."""
        from .abi import MPC_TILE
        tiles = -(-n_cand // MPC_TILE)
        out = torch.empty((tiles, n_steps, 2, MPC_TILE), dtype=torch.float64, device=self.device)
        st = self.lib.mpc_sample_controls_tiled(
            v_grid.data_ptr(), v_grid.numel(), beta_grid.data_ptr(), beta_grid.numel(),
            n_cand, n_steps, int(seed) & 0xFFFFFFFFFFFFFFFF, int(index_base), int(const_prefix),
            out.data_ptr(), _stream_ptr())
        native.check(st, "mpc_sample_controls_tiled")
        return out


def tiled_to_soa(tiles, n_cand):
    """(v, beta) step-major [n_steps, n_cand] copies of a tiled control tensor
    [tiles, n_steps, 2, MPC_TILE] (same device)."""
    t, ns = tiles.shape[0], tiles.shape[1]
    soa = tiles.permute(2, 1, 0, 3).reshape(2, ns, t * tiles.shape[3])[:, :, :n_cand]
    return soa[0].contiguous(), soa[1].contiguous()


def soa_to_tiled(v, beta):
    """The tiled tensor [tiles, n_steps, 2, MPC_TILE] of SoA controls (the last
    tile padded with copies of the last candidate)."""
    from .abi import MPC_TILE
    ns, n = v.shape
    tiles = -(-n // MPC_TILE)
    pad = tiles * MPC_TILE - n
    vb = torch.stack([v, beta])                                  # [2, ns, n]
    if pad:
        vb = torch.cat([vb, vb[:, :, -1:].expand(2, ns, pad)], dim=2)
    return vb.reshape(2, ns, tiles, MPC_TILE).permute(2, 1, 0, 3).contiguous()


def fulltree_argmin(engine, problem, v_grid, beta_grid, incumbent, integrator="qk21", shard=0,
                    n_shards=1):
    """Full-tree MPC step (run_math_model.py:133-228): S1^3 leaves from the
    device grids v_grid [|V|], beta_grid [|B|] (fp64 tensors on the engine's
    device); this call evaluates leaf shard `shard` of `n_shards`.  Returns
    the device result buffer (uint8[FT_RESULT_BYTES])."""
    from .abi import FT_RESULT_BYTES
    lib = engine.lib
    nv, nb = v_grid.numel(), beta_grid.numel()
    ws = engine._workspace(lib.mpc_fulltree_workspace_bytes(nv, nb))
    out = torch.empty(FT_RESULT_BYTES, dtype=torch.uint8, device=engine.device)
    st = lib.mpc_fulltree_argmin(ctypes.byref(problem), v_grid.data_ptr(), nv,
                                 beta_grid.data_ptr(), nb, float(incumbent),
                                 _integ(integrator), int(shard), int(n_shards), ws.data_ptr(),
                                 ws.numel(), out.data_ptr(), _stream_ptr())
    native.check(st, "mpc_fulltree_argmin")
    return out


def fulltree_argmin_batched(engine, problems_dev, incumbents_dev, L, t_a, t_b, v_grid,
                            beta_grid, integrator="qk21", out=None):
    """R robots' full trees (one per run_math_model episode, lockstep):
    problems_dev uint8[R * sizeof(mpc_fulltree_problem_t)], incumbents_dev
    float64[R]; returns the device results uint8[R * FT_RESULT_BYTES]."""
    from .abi import FT_RESULT_BYTES, MpcFulltreeProblem
    lib = engine.lib
    R = problems_dev.numel() // ctypes.sizeof(MpcFulltreeProblem)
    nv, nb = v_grid.numel(), beta_grid.numel()
    ws = engine._workspace(lib.mpc_fulltree_batched_workspace_bytes(R, nv, nb))
    if out is None:
        out = torch.empty(R * FT_RESULT_BYTES, dtype=torch.uint8, device=engine.device)
    st = lib.mpc_fulltree_argmin_batched(
        problems_dev.data_ptr(), incumbents_dev.data_ptr(), R, float(L), float(t_a),
        float(t_b), v_grid.data_ptr(), nv, beta_grid.data_ptr(), nb, _integ(integrator),
        ws.data_ptr(), ws.numel(), out.data_ptr(), _stream_ptr())
    native.check(st, "mpc_fulltree_argmin_batched")
    return out


def fulltree_results(out_dev):
    from .abi import FT_RESULT_BYTES, MpcFulltreeResult
    raw = out_dev.cpu().numpy().tobytes()
    return [MpcFulltreeResult.from_buffer_copy(raw[i:i + FT_RESULT_BYTES])
            for i in range(0, len(raw), FT_RESULT_BYTES)]


def fulltree_result(out_dev):
    from .abi import MpcFulltreeResult
    return MpcFulltreeResult.from_buffer_copy(out_dev.cpu().numpy().tobytes())


def problems_to_device(problems, device):
    """Pack a list of MpcProblem into a device byte tensor (mpc_problem_t[R])."""
    arr = (MpcProblem * len(problems))(*problems)
    host = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
    return host.to(device)


def results_from_device(out_dev):
    raw = out_dev.cpu().numpy().tobytes()
    return [MpcResult.from_buffer_copy(raw[i:i + RESULT_BYTES])
            for i in range(0, len(raw), RESULT_BYTES)]
