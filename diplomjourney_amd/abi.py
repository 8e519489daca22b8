"""ctypes mirror of include/mpc_rollout.h (structs, constants, status codes).

Kept in one place so the product binding (`native.py`) and the test-side
oracle binding agree on the byte layout.  Layout is checked against the C
compiler's sizeof/offsetof in tests/test_abi.py.
"""
import ctypes

MPC_MAX_STEPS = 32

MPC_OK = 0
MPC_ERR_ARG = -1
MPC_ERR_WORKSPACE = -2
MPC_ERR_HIP = -3
MPC_ERR_UNSUPPORTED = -4

MPC_INTEG_QK21 = 0
MPC_INTEG_RECT = 1

MPC_HEADING_ROTATE = 0x100
MPC_HEADING_CUMULATIVE = 0x200

# integrator argument of the C ABI: QUADPACK-exact or exact integral, each
# with the heading evaluated directly (reference formula) or by rotation
# control layout flag OR'ed into the integrator of the chained / P2P entries
# (include/mpc_rollout.h MPC_LAYOUT_TILED): tile t of MPC_TILE candidates holds
# per step its MPC_TILE v values then its MPC_TILE beta values
MPC_LAYOUT_TILED = 0x400
MPC_TILE = 512

INTEGRATORS = {"qk21": MPC_INTEG_QK21, "rect": MPC_INTEG_RECT,
               "qk21+rot": MPC_INTEG_QK21 | MPC_HEADING_ROTATE,
               "rect+rot": MPC_INTEG_RECT | MPC_HEADING_ROTATE,
               # rotation from the identity, start pose applied last (chained steps)
               "rect+cum": MPC_INTEG_RECT | MPC_HEADING_CUMULATIVE}


class MpcProblem(ctypes.Structure):
    """mpc_problem_t: one robot at one MPC step (math_model_tree.py:278-306)."""
    _fields_ = [
        ("x", ctypes.c_double), ("y", ctypes.c_double), ("phi", ctypes.c_double),
        ("x_t", ctypes.c_double), ("y_t", ctypes.c_double),
        ("x_0", ctypes.c_double), ("y_0", ctypes.c_double),
        ("L", ctypes.c_double),
        ("t_a", ctypes.c_double), ("t_b", ctypes.c_double),
    ]

    def as_tuple(self):
        return tuple(getattr(self, n) for n, _ in self._fields_)


class MpcResult(ctypes.Structure):
    """mpc_result_t: the selected candidate and its per-step states."""
    _fields_ = [
        ("cost", ctypes.c_double),
        ("index", ctypes.c_int64),
        ("found", ctypes.c_int32),
        ("n_steps", ctypes.c_int32),
        ("v", ctypes.c_double),
        ("beta", ctypes.c_double),
        ("traj", (ctypes.c_double * 3) * MPC_MAX_STEPS),
    ]

    def trajectory(self):
        return [[self.traj[s][k] for k in range(3)] for s in range(self.n_steps)]

    def as_dict(self):
        return {"cost": self.cost, "index": self.index, "found": bool(self.found),
                "n_steps": self.n_steps, "v": self.v, "beta": self.beta,
                "traj": self.trajectory()}


class MpcCandidate(ctypes.Structure):
    """mpc_candidate_t: one rank's best candidate (the exchange's payload)."""
    _fields_ = [("cost", ctypes.c_double), ("index", ctypes.c_int64),
                ("n_steps", ctypes.c_int32), ("reserved_", ctypes.c_int32),
                ("v", ctypes.c_double * MPC_MAX_STEPS), ("beta", ctypes.c_double * MPC_MAX_STEPS)]


class MpcEpisodeConfig(ctypes.Structure):
    """mpc_episode_config_t: the device-resident math_mpc loop's constants."""
    _fields_ = [(n, ctypes.c_double) for n in (
        "start_x", "start_y", "start_phi", "start_v", "start_beta", "target_x", "target_y",
        "L", "delta_t", "eps", "v_max", "v_min", "delta_v", "ratio_v", "delta_beta",
        "ratio_beta", "beta_bound", "radius_u_turn", "turn_distance", "event_target_x",
        "event_target_y", "incumbent0")] + [(n, ctypes.c_int32) for n in (
        "p_turn_right", "p_turn_left", "p_new_target", "slow_new_target", "slow_turn",
        "max_steps", "enumerate", "stop_rule")] + [("seed", ctypes.c_uint64)]


# mpc_episode_log_t.status bits (include/mpc_rollout.h)
MPC_EP_STALE, MPC_EP_STUCK, MPC_EP_BREAK, MPC_EP_EVENT, MPC_EP_ARRIVED, MPC_EP_LIMIT = (
    1, 2, 4, 8, 16, 32)
MPC_EP_NO_TRAJ = 64     # full-tree episodes: the first call found no winning leaf


class MpcFulltreeEpisodeConfig(ctypes.Structure):
    """mpc_fulltree_episode_config_t: one run_math_model.py episode (:231-280)."""
    _fields_ = [(n, ctypes.c_double) for n in (
        "x_0", "y_0", "phi_0", "x_t", "y_t", "atan_target", "incumbent0")] + [
        ("max_calls", ctypes.c_int32), ("reserved_", ctypes.c_int32)]


class MpcEpisodeLog(ctypes.Structure):
    """mpc_episode_log_t: one MPC step of the device-resident episode."""
    _fields_ = [("step", ctypes.c_int64), ("index", ctypes.c_int64), ("p", ctypes.c_int32),
                ("episode", ctypes.c_int32), ("found", ctypes.c_int32),
                ("status", ctypes.c_int32)] + [(n, ctypes.c_double) for n in (
                    "cost", "x", "y", "phi", "v", "beta")]


class MpcEpisodesProgress(ctypes.Structure):
    """mpc_episodes_progress_t: one robot of the batched device episodes."""
    _fields_ = [("calls", ctypes.c_int32), ("stop", ctypes.c_int32),
                ("candidates", ctypes.c_int64)]


class MpcFulltreeProblem(ctypes.Structure):
    """mpc_fulltree_problem_t: one full-tree MPC step (run_math_model.py:133-156)."""
    _fields_ = [(n, ctypes.c_double) for n in
                ("x", "y", "phi", "x_t", "y_t", "x_0", "y_0", "atan_target", "L", "t_a",
                 "t_b")]


class MpcFulltreeResult(ctypes.Structure):
    """mpc_fulltree_result_t: the first strict-minimum leaf and its three layers."""
    _fields_ = [
        ("cost", ctypes.c_double),
        ("leaf", ctypes.c_int64),
        ("found", ctypes.c_int32),
        ("s1", ctypes.c_int32),
        ("k", ctypes.c_int64 * 3),
        ("v", ctypes.c_double * 3),
        ("beta", ctypes.c_double * 3),
        ("traj", (ctypes.c_double * 3) * 3),
    ]

    def trajectory(self):
        return [[self.traj[i][k] for k in range(3)] for i in range(3)]


RESULT_BYTES = ctypes.sizeof(MpcResult)
CANDIDATE_BYTES = ctypes.sizeof(MpcCandidate)
IPC_HANDLE_BYTES = 64   # MPC_IPC_HANDLE_BYTES (hipIpcMemHandle_t)
FT_RESULT_BYTES = ctypes.sizeof(MpcFulltreeResult)
LOG_BYTES = ctypes.sizeof(MpcEpisodeLog)
PROGRESS_BYTES = ctypes.sizeof(MpcEpisodesProgress)
PROBLEM_BYTES = ctypes.sizeof(MpcProblem)

STATUS_TEXT = {
    MPC_OK: "ok",
    MPC_ERR_ARG: "invalid argument",
    MPC_ERR_WORKSPACE: "workspace too small",
    MPC_ERR_HIP: "HIP runtime error",
    MPC_ERR_UNSUPPORTED: "unsupported option",
}


class MpcError(RuntimeError):
    def __init__(self, status, where=""):
        self.status = status
        super().__init__(f"{where}: status {status} ({STATUS_TEXT.get(status, 'unknown')})")


def result_from_bytes(buf):
    """Decode one mpc_result_t from a bytes-like object (e.g. a CPU uint8 tensor)."""
    return MpcResult.from_buffer_copy(bytes(buf))


def make_problem(x, y, phi, x_t, y_t, x_0, y_0, L, t_a, t_b):
    return MpcProblem(float(x), float(y), float(phi), float(x_t), float(y_t),
                      float(x_0), float(y_0), float(L), float(t_a), float(t_b))
