"""Builds and loads the host test harnesses (trig_harness.cpp, replica_harness.cpp)."""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
BUILD = os.path.join(REPO, "oracle", "_build")
_P = ctypes.c_void_p


def _build(name, cmd):
    out = os.path.join(BUILD, f"lib{name}.so")
    src = os.path.join(HERE, f"{name}.cpp")
    deps = [src, os.path.join(REPO, "diplomjourney_amd", "csrc", "mpc_trig.h"),
            os.path.join(REPO, "diplomjourney_amd", "csrc", "mpc_device.h")]
    if not os.path.exists(out) or any(os.path.getmtime(d) > os.path.getmtime(out) for d in deps):
        os.makedirs(BUILD, exist_ok=True)
        subprocess.run(cmd + ["-o", out, src], check=True)
    return ctypes.CDLL(out)


def trig_lib():
    L = _build("trig_harness", ["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fPIC",
                                "-shared"])
    L.trig_eval.argtypes = [_P, ctypes.c_int64, _P, _P, _P]
    L.trig_tan_small.argtypes = [_P, ctypes.c_int64, _P]
    return L


def trig_eval(x):
    x = np.ascontiguousarray(x, dtype=np.float64)
    n = len(x)
    t, s, c = np.empty(n), np.empty(n), np.empty(n)
    trig_lib().trig_eval(x.ctypes.data_as(_P), n, t.ctypes.data_as(_P), s.ctypes.data_as(_P),
                         c.ctypes.data_as(_P))
    return t, s, c


def tan_small(x):
    x = np.ascontiguousarray(x, dtype=np.float64)
    t = np.empty(len(x))
    trig_lib().trig_tan_small(x.ctypes.data_as(_P), len(x), t.ctypes.data_as(_P))
    return t


def replica_lib():
    from diplomjourney_amd.abi import MpcProblem
    L = _build("replica_harness", ["/opt/rocm/bin/hipcc", "-O2", "-std=c++17",
                                   "-ffp-contract=off", "-fPIC", "-shared", "--cuda-host-only",
                                   "-x", "hip", "-I", os.path.join(REPO, "include")])
    L.replica_rollout.argtypes = [ctypes.POINTER(MpcProblem), _P, _P, ctypes.c_int64,
                                  ctypes.c_int32, ctypes.c_int32, _P, _P]
    L.replica_set_rcp_table.argtypes = [_P, _P, ctypes.c_int64]
    L.replica_rcp_misses.restype = ctypes.c_int64
    L.replica_tan_q.argtypes = [_P, ctypes.c_int64, _P]
    return L


def device_rcp(q):
    """The GPU's reciprocal estimates of q (mpc_rcp_estimate)."""
    import torch
    from diplomjourney_amd import native
    qd = torch.as_tensor(np.ascontiguousarray(q, dtype=np.float64), device="cuda")
    rd = torch.empty_like(qd)
    native.check(native.lib().mpc_rcp_estimate(qd.data_ptr(), rd.data_ptr(), qd.numel(), None),
                 "mpc_rcp_estimate")
    torch.cuda.synchronize()
    return rd.cpu().numpy()


def replica_rollout(problem, v_sc, b_sc, integ="rect", device_estimates=False):
    """Host replica of the kernel arithmetic -> (states [N,3,C], costs [C]).
    device_estimates: the steering tangent's reciprocal estimates come from
    the GPU (every denominator of b_sc), so the result is the device's bit for
    bit; otherwise the host's 1.0 / q (within tolerances of it)."""
    from diplomjourney_amd.abi import INTEGRATORS
    v_sc = np.ascontiguousarray(v_sc, dtype=np.float64)
    b_sc = np.ascontiguousarray(b_sc, dtype=np.float64)
    ns, n = v_sc.shape
    states, costs = np.empty((ns, 3, n)), np.empty(n)
    L = replica_lib()
    if device_estimates:
        beta = np.unique(b_sc)
        q = np.empty_like(beta)
        L.replica_tan_q(beta.ctypes.data_as(_P), len(beta), q.ctypes.data_as(_P))
        q = np.unique(q)
        r = device_rcp(q)
        L.replica_set_rcp_table(q.ctypes.data_as(_P), r.ctypes.data_as(_P), len(q))
    try:
        L.replica_rollout(ctypes.byref(problem), v_sc.ctypes.data_as(_P),
                          b_sc.ctypes.data_as(_P), n, ns, INTEGRATORS[integ],
                          states.ctypes.data_as(_P), costs.ctypes.data_as(_P))
        if device_estimates:
            assert L.replica_rcp_misses() == 0, "a denominator without its device estimate"
    finally:
        if device_estimates:
            L.replica_set_rcp_table(None, None, 0)
    return states, costs
