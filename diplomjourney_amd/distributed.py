"""Candidate sharding and the per-MPC-step winner exchange.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI).
Rank g owns the contiguous candidate range [g*C/G, (g+1)*C/G); its kernel
reports global indices (index_base), so the lowest-index tie-break is the same
as on one device and in the reference's ascending scan.

RCCL has no (min, index) reduction, so every exchange is ONE all_gather
followed by the lexicographic (cost, global index) selection on every rank —
semantically the north star's all-reduce(min+index):
  * the device-resident chained step (DeviceEpisode(exchange=True,
    chain=True), the bench's N > 1 path): `gather_bytes` of each rank's
    536-byte mpc_candidate_t (cost, global index, the candidate's N
    controls); the NEXT launch's block 0 selects the winner and re-rolls it
    from the gathered controls (mpc_episode.h advance_from_candidates);
  * the generic per-call path (Episode, the drop-in's shards):
    `exchange_winner` = all_gather of the 808-byte mpc_result_t records
    (winner trajectory included) + k_select_winner.
Either payload is G x (536 | 808) B: pure latency over xGMI.  RCCL with more
than one rank has not yet run on hardware in this repo's tests (1-rank RCCL
groups, gloo ranks sharing a GPU, and an RCCL clique of one GPU from the C
host are what the tests exercise).
"""
import math

import torch
import torch.distributed as dist

from .abi import RESULT_BYTES, MpcResult


def shard_range(n_total, rank, world):
    """Contiguous [lo, hi) of candidate indices owned by `rank`."""
    base, rem = divmod(n_total, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def gather_results(local_out, group=None):
    """all_gather of one uint8[RESULT_BYTES] record per rank -> uint8[world*RESULT_BYTES].

    RCCL (backend "nccl") gathers device memory directly.  A gloo group
    (CPU tests, or rehearsing several ranks on one GPU) stages through host
    memory."""
    world = dist.get_world_size(group)
    if local_out.is_cuda and dist.get_backend(group) == "gloo":
        host = gather_results(local_out.cpu(), group)
        return host.to(local_out.device)
    gathered = torch.empty(world * RESULT_BYTES, dtype=torch.uint8, device=local_out.device)
    dist.all_gather_into_tensor(gathered, local_out, group=group)
    return gathered


def _key(res):
    """Total order used on device (mpc_device.h cost_key): non-finite or
    missing winners last, then cost, then global index."""
    if res.index < 0 or not (res.cost < math.inf):
        return (1, 0.0, 0)
    return (0, res.cost + 0.0, res.index)


def select_winner_host(records, incumbent=math.inf):
    """Host restatement of k_select_winner for CPU process groups (gloo) and
    tests: records is a list of MpcResult (or a bytes blob of them)."""
    if isinstance(records, (bytes, bytearray, memoryview)):
        raw = bytes(records)
        records = [MpcResult.from_buffer_copy(raw[i:i + RESULT_BYTES])
                   for i in range(0, len(raw), RESULT_BYTES)]
    best = min(range(len(records)), key=lambda r: _key(records[r]))
    out = MpcResult.from_buffer_copy(bytes(records[best]))
    out.found = int(_key(out)[0] == 0 and out.cost < incumbent)
    return out


def exchange_winner(engine, local_out, incumbent=math.inf, group=None):
    """Device path: all_gather (RCCL) + on-device selection into engine.result."""
    gathered = gather_results(local_out, group)
    return engine.select_winner(gathered, incumbent=incumbent)


def select_fulltree(records, incumbent=math.inf):
    """Winner over the per-shard full-tree results (MpcFulltreeResult list or
    the all_gather'ed bytes): lexicographic (cost, global leaf) minimum, as
    the reference's single scan over j; `found` against the incumbent."""
    from .abi import FT_RESULT_BYTES, MpcFulltreeResult
    if isinstance(records, (bytes, bytearray, memoryview)):
        raw = bytes(records)
        records = [MpcFulltreeResult.from_buffer_copy(raw[i:i + FT_RESULT_BYTES])
                   for i in range(0, len(raw), FT_RESULT_BYTES)]

    def key(r):
        if r.leaf < 0 or not (r.cost < math.inf):
            return (1, 0.0, 0)
        return (0, r.cost + 0.0, r.leaf)

    best = min(records, key=key)
    out = MpcFulltreeResult.from_buffer_copy(bytes(best))
    out.found = int(key(out)[0] == 0 and out.cost < incumbent)
    return out


def gather_bytes(local, group=None):
    """all_gather of one uint8 record per rank (RCCL on device tensors; gloo
    groups stage through host memory) -> uint8[world * len]."""
    world = dist.get_world_size(group)
    if local.is_cuda and dist.get_backend(group) == "gloo":
        return gather_bytes(local.cpu(), group).to(local.device)
    out = torch.empty(world * local.numel(), dtype=torch.uint8, device=local.device)
    dist.all_gather_into_tensor(out, local, group=group)
    return out


def gather_into(out, local, group=None):
    """all_gather of one uint8 record per rank into the preallocated `out`
    (uint8[world * len]) on the current stream (RCCL; gloo stages through
    host memory)."""
    if local.is_cuda and dist.get_backend(group) == "gloo":
        out.copy_(gather_bytes(local.cpu(), group), non_blocking=True)
        return out
    dist.all_gather_into_tensor(out, local, group=group)
    return out
