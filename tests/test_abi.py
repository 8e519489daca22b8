"""The C-ABI library: builds, loads, exports every symbol include/mpc_rollout.h
declares, agrees with the ctypes struct layout, and validates arguments
before touching the GPU.  CPU only (no compute calls)."""
import ctypes
import os
import re
import subprocess

import pytest

from diplomjourney_amd import abi, native

HEADER = native.HEADER


def _declared():
    """The functions the header declares for the library to export (its static
    inline helpers, defined in the header itself, excluded)."""
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    inline = set(re.findall(r"static\s+inline\s+[a-z_0-9]+\s+(mpc_[a-z_0-9]+)\s*\(", text))
    return set(re.findall(r"\b(mpc_[a-z_0-9]+)\s*\(", text)) - inline


@pytest.fixture(scope="module")
def so():
    if native.needs_build():
        native.build()
    return ctypes.CDLL(native.LIB_PATH)


def test_exports_match_header(so):
    declared = _declared()
    assert declared == set(native.EXPORTS)
    for name in declared:
        assert hasattr(so, name), name


def test_binding_loads():
    L = native.lib()
    assert b"gfx950" in L.mpc_version()
    assert L.mpc_strerror(abi.MPC_ERR_WORKSPACE) == b"workspace too small"


def test_struct_layout_matches_c(tmp_path):
    src = tmp_path / "layout.c"
    src.write_text(
        '#include <stdio.h>\n#include <stddef.h>\n#include "mpc_rollout.h"\n'
        "int main(void){printf(\"%zu %zu %zu %zu %zu %zu\\n\", sizeof(mpc_problem_t),"
        " sizeof(mpc_result_t), offsetof(mpc_result_t, index), offsetof(mpc_result_t, found),"
        " offsetof(mpc_result_t, v), offsetof(mpc_result_t, traj)); return 0;}\n")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.dirname(HEADER), "-o", str(exe), str(src)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True,
                                          check=True).stdout.split()]
    R = abi.MpcResult
    assert got == [ctypes.sizeof(abi.MpcProblem), ctypes.sizeof(R), R.index.offset,
                   R.found.offset, R.v.offset, R.traj.offset]


def test_episode_struct_layouts_match_c(tmp_path):
    """mpc_episode_config_t (incl. stop_rule), mpc_episode_log_t and
    mpc_episodes_progress_t: the ctypes mirrors equal the C layouts."""
    src = tmp_path / "layout2.c"
    src.write_text(
        '#include <stdio.h>\n#include <stddef.h>\n#include "mpc_rollout.h"\n'
        "int main(void){printf(\"%zu %zu %zu %zu %zu %zu %zu\\n\", sizeof(mpc_episode_config_t),"
        " offsetof(mpc_episode_config_t, stop_rule), offsetof(mpc_episode_config_t, seed),"
        " sizeof(mpc_episode_log_t), sizeof(mpc_episodes_progress_t),"
        " offsetof(mpc_episodes_progress_t, stop), offsetof(mpc_episodes_progress_t, candidates));"
        " return 0;}\n")
    exe = tmp_path / "layout2"
    subprocess.run(["gcc", "-I", os.path.dirname(HEADER), "-o", str(exe), str(src)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True,
                                          check=True).stdout.split()]
    C, P = abi.MpcEpisodeConfig, abi.MpcEpisodesProgress
    assert got == [ctypes.sizeof(C), C.stop_rule.offset, C.seed.offset,
                   ctypes.sizeof(abi.MpcEpisodeLog), ctypes.sizeof(P), P.stop.offset,
                   P.candidates.offset]


def test_batched_episodes_argument_validation_without_gpu():
    """mpc_episodes_*: sizes and rejected arguments, before any HIP call."""
    from diplomjourney_amd.episode import reference_episode_config
    L = native.lib()
    assert L.mpc_episodes_state_bytes(0) == 0
    n1 = L.mpc_episodes_state_bytes(1)
    assert L.mpc_episodes_state_bytes(1000) > 1000 * ctypes.sizeof(abi.MpcEpisodeConfig) > n1 > 0
    fake = ctypes.c_void_p(0x1000)
    cfg = reference_episode_config()
    bad = reference_episode_config()
    bad.stop_rule = 2
    arr = (abi.MpcEpisodeConfig * 2)(cfg, bad)
    assert L.mpc_episodes_reset(ctypes.byref(arr), 2, fake, None) == abi.MPC_ERR_ARG
    assert L.mpc_episodes_reset(None, 1, fake, None) == abi.MPC_ERR_ARG
    assert L.mpc_episodes_reset(ctypes.byref(arr), 0, fake, None) == abi.MPC_ERR_ARG
    assert L.mpc_episodes_run(None, 1, 3, 0, 1, None, 0, None, None) == abi.MPC_ERR_ARG
    assert L.mpc_episodes_run(fake, 1, 0, 0, 1, None, 0, None, None) == abi.MPC_ERR_ARG
    assert L.mpc_episodes_run(fake, 1, 3, 0, 1, fake, 0, None, None) == abi.MPC_ERR_ARG
    assert L.mpc_episodes_run(fake, 1, 3, 7, 1, None, 0, None, None) == abi.MPC_ERR_UNSUPPORTED
    assert L.mpc_episodes_run(fake, 1, 3, 0, 0, None, 0, None, None) == abi.MPC_OK   # nothing


def test_persistent_run_argument_validation_without_gpu():
    """mpc_episode_run: workspace size and rejected arguments, before any HIP
    call (epoch 0 or an epoch range past 2^32 - 1, no steps, a horizon out of
    range, a heading mode other than rect+cum, misaligned or mismatched
    tiled controls, too small a workspace)."""
    from diplomjourney_amd.episode import reference_episode_config
    L = native.lib()
    n, ns = 20_000, 10
    tiles = -(-n // 512)
    wsb = L.mpc_episode_run_workspace_bytes(n)
    assert wsb == 256 + 2 * tiles * 16 and L.mpc_episode_run_workspace_bytes(1) == 0
    cfg = reference_episode_config()
    fake = 0x10000
    V = (ctypes.c_void_p * 2)(fake, fake + 16 * n)
    B = (ctypes.c_void_p * 2)(fake + 8 * n * ns, fake + 24 * n)
    cum = abi.INTEGRATORS["rect+cum"]

    def run(e0=1, k=2, nsteps=ns, integ=cum, v=V, b=B, ws=wsb, nc=n):
        return L.mpc_episode_run(ctypes.byref(cfg), ctypes.c_void_p(fake), e0, v, b, k, nc,
                                 nsteps, 0, integ, ctypes.c_void_p(fake), ws, ctypes.c_void_p(fake),
                                 None, 0, None)

    assert run(e0=0) == abi.MPC_ERR_ARG
    assert run(e0=0xFFFFFFFF) == abi.MPC_ERR_ARG          # epochs would wrap to 0
    assert run(k=0) == abi.MPC_ERR_ARG
    assert run(nsteps=0) == abi.MPC_ERR_ARG
    assert run(nc=1) == abi.MPC_ERR_ARG
    assert run(integ=abi.INTEGRATORS["rect+rot"]) == abi.MPC_ERR_UNSUPPORTED
    Bm = (ctypes.c_void_p * 2)(fake + 8, fake + 24 * n)   # misaligned beta row
    assert run(b=Bm) == abi.MPC_ERR_UNSUPPORTED
    Bt = (ctypes.c_void_p * 2)(fake + 8 * 512, fake + 8)  # tiled: beta must be v + 512
    assert run(integ=cum | abi.MPC_LAYOUT_TILED, b=Bt) == abi.MPC_ERR_UNSUPPORTED
    assert run(ws=wsb - 1) == abi.MPC_ERR_WORKSPACE


def test_workspace_sizes():
    L = native.lib()
    assert L.mpc_workspace_bytes(1, 3) == 16
    assert L.mpc_workspace_bytes(10**7, 12) == 2048 * 16   # capped grid
    assert L.mpc_batched_workspace_bytes(4, 10_000, 8) == 4 * 40 * 16


def test_argument_validation_without_gpu():
    """Invalid arguments are rejected before any HIP call."""
    L = native.lib()
    p = abi.make_problem(0, 0, 0, 2, 3, 0, 0, 0.5, 0.05, 0.1)
    fake = ctypes.c_void_p(0x1000)
    args = dict(v=fake, b=fake, n=100, ns=3, base=0, inc=1e300, integ=0, st=None, ws=fake,
                wsb=1 << 20, out=fake)

    def call(**kw):
        a = {**args, **kw}
        return L.mpc_rollout_argmin(ctypes.byref(p), a["v"], a["b"], a["n"], a["ns"], a["base"],
                                    a["inc"], a["integ"], a["st"], a["ws"], a["wsb"], a["out"],
                                    None)

    assert call(n=0) == abi.MPC_ERR_ARG
    assert call(ns=0) == abi.MPC_ERR_ARG
    assert call(ns=abi.MPC_MAX_STEPS + 1) == abi.MPC_ERR_ARG
    assert call(v=None) == abi.MPC_ERR_ARG
    assert call(out=None) == abi.MPC_ERR_ARG
    assert call(base=-1) == abi.MPC_ERR_ARG
    assert call(integ=7) == abi.MPC_ERR_UNSUPPORTED
    assert call(wsb=8) == abi.MPC_ERR_WORKSPACE
    assert L.mpc_rollout_argmin(None, fake, fake, 10, 3, 0, 1.0, 0, None, fake, 1 << 20, fake,
                                None) == abi.MPC_ERR_ARG
    assert L.mpc_select_winner(None, 1, 1.0, fake, None) == abi.MPC_ERR_ARG
    assert L.mpc_sample_controls(fake, 3, fake, 4, 10, 3, 1, 0, 1, fake, fake, 5,
                                 None) == abi.MPC_ERR_ARG  # ld < n_cand
    assert L.mpc_rollout_argmin_batched(fake, None, 0, fake, fake, 10, 3, 0, fake, 1 << 20,
                                        fake, None) == abi.MPC_ERR_ARG
    # the verification probe: nothing to do, a negative count, missing arrays
    assert L.mpc_rcp_estimate(None, None, 0, None) == abi.MPC_OK
    assert L.mpc_rcp_estimate(fake, fake, -1, None) == abi.MPC_ERR_ARG
    assert L.mpc_rcp_estimate(None, fake, 4, None) == abi.MPC_ERR_ARG


def test_no_cpu_fallback(monkeypatch, tmp_path):
    """The product binding raises when the HIP library is absent."""
    monkeypatch.setattr(native, "_lib", None)
    monkeypatch.setattr(native, "LIB_PATH", str(tmp_path / "missing.so"))
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        native.lib()


def test_p2p_exchange_argument_validation_without_gpu():
    """mpc_mailbox_* / mpc_ipc_* / mpc_episode_p2p_*: sizes and rejected
    arguments, before any HIP call."""
    from diplomjourney_amd.episode import reference_episode_config
    L = native.lib()
    assert L.mpc_mailbox_bytes(0) == 0 and L.mpc_mailbox_bytes(33) == 0
    one, eight = L.mpc_mailbox_bytes(1), L.mpc_mailbox_bytes(8)
    # header (32 peer pointers, rank, world, 32 ping words; 256-B padded), then
    # two slots of one candidate per rank, each 8-B word as a 16-B tagged granule
    rec = abi.CANDIDATE_BYTES * 2
    hdr = one - 2 * rec
    assert eight - one == 2 * 7 * rec and hdr % 256 == 0 and hdr >= 32 * 8 * 2 + 8
    out = ctypes.c_void_p()
    assert L.mpc_mailbox_alloc(0, 1, ctypes.byref(out)) == abi.MPC_ERR_ARG
    assert L.mpc_mailbox_alloc(2, 1, None) == abi.MPC_ERR_ARG
    assert L.mpc_mailbox_free(None) == abi.MPC_ERR_ARG
    assert L.mpc_ipc_handle(None, None) == abi.MPC_ERR_ARG
    assert L.mpc_ipc_open(None, ctypes.byref(out)) == abi.MPC_ERR_ARG
    assert L.mpc_ipc_close(None) == abi.MPC_ERR_ARG
    f = ctypes.c_void_p(0x1000)
    g = ctypes.c_void_p(0x2000)
    peers = (ctypes.c_void_p * 2)(f, g)
    assert L.mpc_mailbox_set_peers(None, 0, 2, peers) == abi.MPC_ERR_ARG
    assert L.mpc_mailbox_set_peers(f, 2, 2, peers) == abi.MPC_ERR_ARG
    assert L.mpc_mailbox_set_peers(f, 1, 2, peers) == abi.MPC_ERR_ARG   # own row != mailbox
    assert L.mpc_mailbox_set_peers(f, 0, 33, peers) == abi.MPC_ERR_ARG
    assert L.mpc_mailbox_ping(None, 1, f, None) == abi.MPC_ERR_ARG
    assert L.mpc_mailbox_ping(f, 0, f, None) == abi.MPC_ERR_ARG
    assert L.mpc_mailbox_ping(f, 1, None, None) == abi.MPC_ERR_ARG
    cfg = reference_episode_config()
    ig = abi.INTEGRATORS["rect+cum"]

    def step(epoch=3, prev=2, mailbox=f, world=2, out_prev=f, ws_prev=f, v_prev=f):
        return L.mpc_episode_p2p_step(ctypes.byref(cfg), f, epoch, prev, f, f, 1024, 10, 0, ig,
                                      f, ws_prev, 1 << 20, v_prev, f, mailbox, world, out_prev,
                                      f, 8, None)
    assert step(epoch=0) == abi.MPC_ERR_ARG
    assert step(prev=1) == abi.MPC_ERR_ARG             # same parity: same mailbox slot
    assert step(mailbox=None) == abi.MPC_ERR_ARG
    assert step(world=0) == abi.MPC_ERR_ARG
    assert step(world=33) == abi.MPC_ERR_ARG
    assert step(out_prev=None) == abi.MPC_ERR_ARG      # a previous step to complete ...
    assert step(ws_prev=None) == abi.MPC_ERR_ARG       # ... from its records
    assert step(v_prev=None) == abi.MPC_ERR_ARG        # ... and controls

    def flush(epoch=3, mailbox=f, world=2, out=f, ws=f):
        return L.mpc_episode_p2p_flush(ctypes.byref(cfg), f, epoch, f, f, 1024, 10, 0, ig, ws,
                                       1 << 20, mailbox, world, out, f, 8, None)
    assert flush(epoch=0) == abi.MPC_ERR_ARG
    assert flush(mailbox=None) == abi.MPC_ERR_ARG
    assert flush(world=0) == abi.MPC_ERR_ARG
    assert flush(out=None) == abi.MPC_ERR_ARG
    assert flush(ws=None) == abi.MPC_ERR_ARG


def test_tiled_layout_argument_validation_without_gpu():
    """MPC_LAYOUT_TILED: accepted only by the chained one-GPU / P2P entries and
    their flush; the tiled buffer's beta must be its base + 512, n_cand even.
    Every rejection happens before any HIP call."""
    from diplomjourney_amd.episode import reference_episode_config
    L = native.lib()
    cfg = reference_episode_config()
    t = abi.MPC_LAYOUT_TILED
    cum = abi.INTEGRATORS["rect+cum"]
    base = ctypes.c_void_p(0x10000)
    b_ok = ctypes.c_void_p(0x10000 + 8 * abi.MPC_TILE)
    b_bad = ctypes.c_void_p(0x20000)
    f = ctypes.c_void_p(0x1000)

    def chain(integ=cum | t, v=base, b=b_ok, n=1024):
        return L.mpc_episode_chain_step(ctypes.byref(cfg), f, 1, 1, v, b, n, 10, 0, integ, f, f,
                                        1 << 24, None, None, f, None, 0, f, 8, None)
    assert chain(b=b_bad) == abi.MPC_ERR_UNSUPPORTED          # beta != base + 512
    assert chain(n=1023) == abi.MPC_ERR_UNSUPPORTED           # two candidates per lane
    assert chain(v=ctypes.c_void_p(0x10008), b=ctypes.c_void_p(0x10008 + 4096)) == \
        abi.MPC_ERR_UNSUPPORTED                               # 16-B aligned base
    assert chain(integ=abi.INTEGRATORS["rect"] | t) == abi.MPC_ERR_UNSUPPORTED   # chained: +cum
    # entries that read SoA controls refuse the flag
    assert L.mpc_episode_partials(f, base, b_ok, 1024, 10, cum | t, f, 1 << 24, None) == \
        abi.MPC_ERR_UNSUPPORTED
    assert L.mpc_episode_exchange_step(ctypes.byref(cfg), f, 1, base, b_ok, 1024, 10, 0, cum | t,
                                       f, 1 << 24, None, 0, f, f, f, 8, None) == \
        abi.MPC_ERR_UNSUPPORTED
    # the flush of a tiled chained step needs the episode update (advance)
    assert L.mpc_episode_finalize(f, base, b_ok, 1024, 10, 0, cum | t, f, 1 << 24, f, None, f,
                                  8, None) == abi.MPC_ERR_UNSUPPORTED
    sink = ctypes.c_void_p(0x40000)
    assert L.mpc_stream_probe_tiled(ctypes.c_void_p(0x10008), 1024, 10, sink, 1 << 30, None) == \
        abi.MPC_ERR_UNSUPPORTED
    assert L.mpc_stream_probe_tiled(base, 1024, 0, sink, 1 << 30, None) == abi.MPC_ERR_ARG
    assert L.mpc_sample_controls_tiled(f, 3, f, 4, 1023, 10, 1, 0, 1, base, None) == \
        abi.MPC_ERR_ARG


def test_tiled_index_header_matches_python(tmp_path):
    """The header's mpc_tiled_index (C) == soa_to_tiled / tiled_to_soa
    (torch, CPU): every candidate and step of a ragged last tile."""
    import torch
    from diplomjourney_amd.expansion import soa_to_tiled, tiled_to_soa
    n, ns = 1300, 3
    src = tmp_path / "ti.c"
    src.write_text(
        '#include <stdio.h>\n#include "mpc_rollout.h"\n'
        "int main(void) { for (int s = 0; s < %d; ++s) for (long c = 0; c < %d; ++c)"
        ' printf("%%ld\\n", (long)mpc_tiled_index(c, s, %d)); return 0; }\n' % (ns, n, ns))
    exe = tmp_path / "ti"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.dirname(HEADER), "-o", str(exe), str(src)],
                   check=True)
    idx = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True,
                                          check=True).stdout.split()]
    v = torch.arange(ns * n, dtype=torch.float64).reshape(ns, n)
    b = -v - 1
    t = soa_to_tiled(v, b)
    flat = t.reshape(-1)
    for s in range(ns):
        for c in range(0, n, 7):
            o = idx[s * n + c]
            assert flat[o] == v[s, c] and flat[o + abi.MPC_TILE] == b[s, c]
    v2, b2 = tiled_to_soa(t, n)
    assert torch.equal(v2, v) and torch.equal(b2, b)
