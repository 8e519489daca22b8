"""ctypes binding of the HIP library libmpc_rollout.so (include/mpc_rollout.h).

The product path has no CPU fallback: if the in-tree library is missing or a
call returns a non-zero status, this module raises.  Device buffers come from
PyTorch-ROCm tensors (`tensor.data_ptr()`), the stream from
`torch.cuda.current_stream().cuda_stream`.  torch is imported first so the
library's libamdhip64.so.7 dependency resolves to the runtime torch already
loaded (one HIP runtime per process).
"""
import ctypes
import os
import subprocess
import sys

from .abi import MpcEpisodeConfig, MpcError, MpcFulltreeProblem, MpcProblem

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
LIB_NAME = "libmpc_rollout.so"
LIB_PATH = os.path.join(PKG_DIR, LIB_NAME)
SRC = os.path.join(PKG_DIR, "csrc", "mpc_rollout.hip")
HEADER = os.path.join(REPO_DIR, "include", "mpc_rollout.h")

# Every symbol include/mpc_rollout.h declares (checked by tests/test_abi.py).
EXPORTS = (
    "mpc_version", "mpc_strerror", "mpc_workspace_bytes", "mpc_rollout_argmin",
    "mpc_rollout_partials", "mpc_rollout_finalize",
    "mpc_batched_workspace_bytes", "mpc_rollout_argmin_batched", "mpc_select_winner",
    "mpc_stream_probe", "mpc_rcp_estimate",
    "mpc_sample_controls", "mpc_episode_state_bytes", "mpc_episode_reset",
    "mpc_episode_expand", "mpc_episode_advance", "mpc_episode_sample", "mpc_episode_partials",
    "mpc_episode_finalize", "mpc_episode_rollout", "mpc_episode_step", "mpc_episode_chain_step",
    "mpc_episode_chain_error", "mpc_episode_exchange_step", "mpc_episode_exchange_flush",
    "mpc_comm_unique_id", "mpc_comm_init_rank", "mpc_comm_init_all", "mpc_comm_destroy",
    "mpc_exchange_allgather", "mpc_exchange_allgather_group",
    "mpc_episode_generate_workspace_bytes", "mpc_episode_generate_step",
    "mpc_fulltree_workspace_bytes", "mpc_fulltree_argmin",
    "mpc_fulltree_batched_workspace_bytes", "mpc_fulltree_argmin_batched",
    "mpc_episodes_state_bytes", "mpc_episodes_reset", "mpc_episodes_run",
    "mpc_episode_exchange_step2", "mpc_episode_exchange_mark",
    "mpc_stream_create_cu_reserved", "mpc_stream_create_cu_share", "mpc_stream_destroy",
    "mpc_mailbox_bytes", "mpc_mailbox_alloc", "mpc_mailbox_free", "mpc_mailbox_set_peers",
    "mpc_mailbox_ping", "mpc_mailbox_clear",
    "mpc_ipc_handle",
    "mpc_ipc_open", "mpc_ipc_close", "mpc_peer_enable", "mpc_episode_p2p_step",
    "mpc_episode_p2p_flush",
    "mpc_fulltree_episodes_state_bytes", "mpc_fulltree_episodes_reset",
    "mpc_fulltree_episodes_run", "mpc_stream_probe_tiled", "mpc_sample_controls_tiled",
    "mpc_episode_run_workspace_bytes", "mpc_episode_run",
)

HIPCC_FLAGS = [
    "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-ldl",
    # One IEEE rounding per reference operator: no a*b+c contraction.
    "-ffp-contract=off",
    "-Wall",
]


def build(verbose=False):
    """Compile csrc/*.hip for gfx950 into the in-tree shared library."""
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc, *HIPCC_FLAGS, "-I", os.path.join(REPO_DIR, "include"), "-o", LIB_PATH, SRC]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    return LIB_PATH


C_HOST_SRC = os.path.join(REPO_DIR, "tests", "c_host", "exchange_episode.cpp")
C_HOST_BIN = os.path.join(REPO_DIR, "tests", "_build", "exchange_episode")


def build_c_host(verbose=False):
    """The test-side C++ host program (tests/c_host): the sharded episode
    through the C ABI and RCCL only, linked against the in-tree library."""
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    os.makedirs(os.path.dirname(C_HOST_BIN), exist_ok=True)
    cmd = [hipcc, "--offload-arch=gfx950", "-O2", "-std=c++17", "-I",
           os.path.join(REPO_DIR, "include"), "-o", C_HOST_BIN, C_HOST_SRC, "-L", PKG_DIR,
           "-lmpc_rollout", "-Wl,-rpath,$ORIGIN/../../diplomjourney_amd"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    return C_HOST_BIN


def needs_build():
    if not os.path.exists(LIB_PATH):
        return True
    lib_m = os.path.getmtime(LIB_PATH)
    srcs = [HEADER] + [os.path.join(PKG_DIR, "csrc", f) for f in os.listdir(os.path.join(PKG_DIR, "csrc"))]
    return any(os.path.getmtime(s) > lib_m for s in srcs)


_lib = None

_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_I64 = ctypes.c_int64
_D = ctypes.c_double


def lib():
    """Load the HIP library (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    import torch  # noqa: F401  (one HIP runtime: torch's libamdhip64.so.7)
    path = LIB_PATH
    if not os.path.exists(path):
        raise RuntimeError(f"{path} is missing: run __graft_entry__.build() "
                           "(the MPC expansion has no CPU fallback)")
    L = ctypes.CDLL(path)
    L.mpc_version.restype = ctypes.c_char_p
    L.mpc_version.argtypes = []
    L.mpc_strerror.restype = ctypes.c_char_p
    L.mpc_strerror.argtypes = [ctypes.c_int]
    L.mpc_workspace_bytes.restype = ctypes.c_size_t
    L.mpc_workspace_bytes.argtypes = [_I64, _I32]
    L.mpc_rollout_argmin.restype = ctypes.c_int
    L.mpc_rollout_argmin.argtypes = [ctypes.POINTER(MpcProblem), _P, _P, _I64, _I32, _I64, _D,
                                     _I32, _P, _P, ctypes.c_size_t, _P, _P]
    L.mpc_rollout_partials.restype = ctypes.c_int
    L.mpc_rollout_partials.argtypes = [ctypes.POINTER(MpcProblem), _P, _P, _I64, _I32, _I32, _P,
                                       _P, ctypes.c_size_t, _P]
    L.mpc_rollout_finalize.restype = ctypes.c_int
    L.mpc_rollout_finalize.argtypes = [ctypes.POINTER(MpcProblem), _P, _P, _I64, _I32, _I64, _D,
                                       _I32, _I32, _P, ctypes.c_size_t, _P, _P]
    L.mpc_batched_workspace_bytes.restype = ctypes.c_size_t
    L.mpc_batched_workspace_bytes.argtypes = [_I32, _I64, _I32]
    L.mpc_rollout_argmin_batched.restype = ctypes.c_int
    L.mpc_rollout_argmin_batched.argtypes = [_P, _P, _I32, _P, _P, _I64, _I32, _I32, _P,
                                             ctypes.c_size_t, _P, _P]
    L.mpc_stream_probe.restype = ctypes.c_int
    L.mpc_stream_probe.argtypes = [_P, _P, _I64, _I32, _P, ctypes.c_size_t, _P]
    L.mpc_stream_probe_tiled.restype = ctypes.c_int
    L.mpc_stream_probe_tiled.argtypes = [_P, _I64, _I32, _P, ctypes.c_size_t, _P]
    L.mpc_sample_controls_tiled.restype = ctypes.c_int
    L.mpc_sample_controls_tiled.argtypes = [_P, _I32, _P, _I32, _I64, _I32, ctypes.c_uint64,
                                            _I64, _I32, _P, _P]
    L.mpc_rcp_estimate.restype = ctypes.c_int
    L.mpc_rcp_estimate.argtypes = [_P, _P, _I64, _P]
    L.mpc_select_winner.restype = ctypes.c_int
    L.mpc_select_winner.argtypes = [_P, _I32, _D, _P, _P]
    L.mpc_sample_controls.restype = ctypes.c_int
    L.mpc_sample_controls.argtypes = [_P, _I32, _P, _I32, _I64, _I32, ctypes.c_uint64, _I64,
                                      _I32, _P, _P, _I64, _P]
    L.mpc_episode_state_bytes.restype = ctypes.c_size_t
    L.mpc_episode_state_bytes.argtypes = []
    L.mpc_episode_reset.restype = ctypes.c_int
    L.mpc_episode_reset.argtypes = [ctypes.POINTER(MpcEpisodeConfig), _P, _P]
    L.mpc_episode_expand.restype = ctypes.c_int
    L.mpc_episode_expand.argtypes = [ctypes.POINTER(MpcEpisodeConfig), _P, _P, _P, _I64, _I32,
                                     _I64, _I32, _P, ctypes.c_size_t, _P, _P]
    L.mpc_episode_advance.restype = ctypes.c_int
    L.mpc_episode_advance.argtypes = [ctypes.POINTER(MpcEpisodeConfig), _P, _P, _I32, _P, _I32,
                                      _P]
    L.mpc_episode_sample.restype = ctypes.c_int
    L.mpc_episode_sample.argtypes = [ctypes.POINTER(MpcEpisodeConfig), _P, _P, _P, _I64, _I32,
                                     _I64, _P]
    L.mpc_episode_partials.restype = ctypes.c_int
    L.mpc_episode_partials.argtypes = [_P, _P, _P, _I64, _I32, _I32, _P, ctypes.c_size_t, _P]
    L.mpc_episode_finalize.restype = ctypes.c_int
    L.mpc_episode_finalize.argtypes = [_P, _P, _P, _I64, _I32, _I64, _I32, _P, ctypes.c_size_t,
                                       _P, ctypes.POINTER(MpcEpisodeConfig), _P, _I32, _P]
    L.mpc_fulltree_workspace_bytes.restype = ctypes.c_size_t
    L.mpc_fulltree_workspace_bytes.argtypes = [_I32, _I32]
    L.mpc_fulltree_argmin.restype = ctypes.c_int
    L.mpc_fulltree_argmin.argtypes = [ctypes.POINTER(MpcFulltreeProblem), _P, _I32, _P, _I32,
                                      ctypes.c_double, _I32, _I32, _I32, _P, ctypes.c_size_t,
                                      _P, _P]
    L.mpc_fulltree_batched_workspace_bytes.restype = ctypes.c_size_t
    L.mpc_fulltree_batched_workspace_bytes.argtypes = [_I32, _I32, _I32]
    L.mpc_fulltree_argmin_batched.restype = ctypes.c_int
    L.mpc_fulltree_argmin_batched.argtypes = [_P, _P, _I32, ctypes.c_double, ctypes.c_double,
                                              ctypes.c_double, _P, _I32, _P, _I32, _I32, _P,
                                              ctypes.c_size_t, _P, _P]
    L.mpc_episode_step.restype = ctypes.c_int
    L.mpc_episode_step.argtypes = L.mpc_episode_finalize.argtypes
    L.mpc_episode_chain_step.restype = ctypes.c_int
    L.mpc_episode_chain_step.argtypes = [ctypes.POINTER(MpcEpisodeConfig), _P, _I32,
                                         ctypes.c_uint32, _P, _P,
                                         _I64, _I32, _I64, _I32, _P, _P, ctypes.c_size_t, _P,
                                         _P, _P, _P, _I32, _P, _I32, _P]
    L.mpc_episode_run_workspace_bytes.restype = ctypes.c_size_t
    L.mpc_episode_run_workspace_bytes.argtypes = [_I64]
    L.mpc_episode_run.restype = ctypes.c_int
    L.mpc_episode_run.argtypes = [ctypes.POINTER(MpcEpisodeConfig), _P, ctypes.c_uint32,
                                  ctypes.POINTER(_P), ctypes.POINTER(_P), _I32, _I64, _I32, _I64,
                                  _I32, _P, ctypes.c_size_t, _P, _P, _I32, _P]
    L.mpc_episode_exchange_step.restype = ctypes.c_int
    L.mpc_episode_exchange_step.argtypes = [ctypes.POINTER(MpcEpisodeConfig), _P, ctypes.c_uint32,
                                            _P, _P, _I64, _I32, _I64, _I32, _P, ctypes.c_size_t,
                                            _P, _I32, _P, _P, _P, _I32, _P]
    L.mpc_episode_exchange_step2.restype = ctypes.c_int
    L.mpc_episode_exchange_step2.argtypes = [
        ctypes.POINTER(MpcEpisodeConfig), _P, ctypes.c_uint32, ctypes.c_uint32, _P, _P, _I64,
        _I32, _I64, _I32, _P, ctypes.c_size_t, _P, _I32, _P, _P, _P, _I32, _P]
    L.mpc_episode_exchange_mark.restype = ctypes.c_int
    L.mpc_episode_exchange_mark.argtypes = [_P, ctypes.c_uint32, _P]
    L.mpc_stream_create_cu_reserved.restype = ctypes.c_int
    L.mpc_stream_create_cu_reserved.argtypes = [_I32, ctypes.POINTER(_P)]
    L.mpc_stream_create_cu_share.restype = ctypes.c_int
    L.mpc_stream_create_cu_share.argtypes = [_I32, _I32, ctypes.POINTER(_P)]
    L.mpc_stream_destroy.restype = ctypes.c_int
    L.mpc_stream_destroy.argtypes = [_P]
    L.mpc_episode_exchange_flush.restype = ctypes.c_int
    L.mpc_episode_exchange_flush.argtypes = [ctypes.POINTER(MpcEpisodeConfig), _P, _I32, _P, _I32,
                                             _P, _P, _I32, _P]
    L.mpc_episode_chain_error.restype = ctypes.c_int
    L.mpc_episode_chain_error.argtypes = [_P, ctypes.POINTER(_I32), _P]
    L.mpc_episode_generate_workspace_bytes.restype = ctypes.c_size_t
    L.mpc_episode_generate_workspace_bytes.argtypes = [_I64, _I32]
    L.mpc_episode_generate_step.restype = ctypes.c_int
    L.mpc_episode_generate_step.argtypes = [ctypes.POINTER(MpcEpisodeConfig), _P, _I64, _I32,
                                            _I64, _I32, _P, ctypes.c_size_t, _P, _P, _I32, _P]
    L.mpc_episode_rollout.restype = ctypes.c_int
    L.mpc_episode_rollout.argtypes = [_P, _P, _P, _I64, _I32, _I64, _I32, _P, ctypes.c_size_t,
                                      _P, ctypes.POINTER(MpcEpisodeConfig), _P, _I32, _P]
    L.mpc_mailbox_bytes.restype = ctypes.c_size_t
    L.mpc_mailbox_bytes.argtypes = [_I32]
    L.mpc_mailbox_alloc.restype = ctypes.c_int
    L.mpc_mailbox_alloc.argtypes = [_I32, _I32, ctypes.POINTER(_P)]
    L.mpc_mailbox_free.restype = ctypes.c_int
    L.mpc_mailbox_free.argtypes = [_P]
    L.mpc_ipc_handle.restype = ctypes.c_int
    L.mpc_ipc_handle.argtypes = [_P, _P]
    L.mpc_ipc_open.restype = ctypes.c_int
    L.mpc_ipc_open.argtypes = [_P, ctypes.POINTER(_P)]
    L.mpc_ipc_close.restype = ctypes.c_int
    L.mpc_ipc_close.argtypes = [_P]
    L.mpc_peer_enable.restype = ctypes.c_int
    L.mpc_peer_enable.argtypes = [_I32]
    L.mpc_mailbox_ping.restype = ctypes.c_int
    L.mpc_mailbox_ping.argtypes = [_P, ctypes.c_uint32, _P, _P]
    L.mpc_mailbox_clear.restype = ctypes.c_int
    L.mpc_mailbox_clear.argtypes = [_P, _I32, _P]
    L.mpc_mailbox_set_peers.restype = ctypes.c_int
    L.mpc_mailbox_set_peers.argtypes = [_P, _I32, _I32, ctypes.POINTER(_P)]
    L.mpc_episode_p2p_step.restype = ctypes.c_int
    L.mpc_episode_p2p_step.argtypes = [
        ctypes.POINTER(MpcEpisodeConfig), _P, ctypes.c_uint32, ctypes.c_uint32, _P, _P, _I64,
        _I32, _I64, _I32, _P, _P, ctypes.c_size_t, _P, _P, _P, _I32, _P, _P, _I32, _P]
    L.mpc_episode_p2p_flush.restype = ctypes.c_int
    L.mpc_episode_p2p_flush.argtypes = [
        ctypes.POINTER(MpcEpisodeConfig), _P, ctypes.c_uint32, _P, _P, _I64, _I32, _I64,
        _I32, _P, ctypes.c_size_t, _P, _I32, _P, _P, _I32, _P]
    L.mpc_episodes_state_bytes.restype = ctypes.c_size_t
    L.mpc_episodes_state_bytes.argtypes = [_I32]
    L.mpc_episodes_reset.restype = ctypes.c_int
    L.mpc_episodes_reset.argtypes = [_P, _I32, _P, _P]
    L.mpc_episodes_run.restype = ctypes.c_int
    L.mpc_episodes_run.argtypes = [_P, _I32, _I32, _I32, _I32, _P, _I32, _P, _P]
    L.mpc_fulltree_episodes_state_bytes.restype = ctypes.c_size_t
    L.mpc_fulltree_episodes_state_bytes.argtypes = [_I32]
    L.mpc_fulltree_episodes_reset.restype = ctypes.c_int
    L.mpc_fulltree_episodes_reset.argtypes = [_P, _I32, _P, _P]
    L.mpc_fulltree_episodes_run.restype = ctypes.c_int
    L.mpc_fulltree_episodes_run.argtypes = [
        _P, _I32, _P, _I32, _P, _I32, ctypes.c_double, ctypes.c_double, ctypes.c_double,
        _I32, _I32, _P, _I32, _P, _P]
    _lib = L
    return L


def check(status, where):
    if status != 0:
        raise MpcError(status, where)
