"""Per-block timeline of the chained step (k_episode_chain): a variant build of
the library with s_memrealtime (100 MHz) stamps patched into a copy of the
sources (the shipped sources carry none), then one chained step among
back-to-back ones, decoded per phase.

    python tools/chain_timeline.py build            # -> tools/tl_variant.so (CPU)
    python tools/chain_timeline.py run N_CAND N [p2p|tiled]   # on the GPU box (p2p: the
                                                    # one-rank P2P exchange form; tiled: the
                                                    # bench default's tiled batches)

Block 0 (completion of step k-1): entry, records loaded + lane minima, wave
arg-min, block winner (after the barrier), winner re-rolled (emit_winner),
episode updated (thread 0), head stored + constants published.
Tile blocks: entry, first control DMAs in flight (pre0), final constants in
hand (after the loop), record stored."""
import ctypes
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VAR = os.path.join(REPO, "tools", "tl_variant.so")   # git-ignored; delete after use (every gpurun call ships it)
NB = 2048 + 1
B0 = ["entry", "records", "wave argmin", "block winner", "controls in LDS", "re-roll",
      "advance", "update", "published", "adv-entry", "finishing", "pre-prepare", "prepared",
      "early pub", "tail done", "t64 early prep", "ew bcast", "ew phase1", "w1 sincos", "l0 pose"]
B0_BASE = 8 * NB   # block 0's stamps follow the tiles' (8 per block)
TILE = ["entry", "DMAs issued", "final consts", "record stored", "costs done", "argmin done"]

STAMP = "__hip_atomic_store(&g_tl[{slot}], __builtin_amdgcn_s_memrealtime(), " \
        "__ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)"


def patch(path, edits):
    s = open(path).read()
    for anchor, new in edits:
        if s.count(anchor) != 1:
            raise SystemExit(f"{os.path.basename(path)}: anchor found {s.count(anchor)}x: {anchor!r}")
        s = s.replace(anchor, new)
    open(path, "w").write(s)


def build():
    d = tempfile.mkdtemp()
    shutil.copytree(os.path.join(REPO, "include"), os.path.join(d, "include"))
    shutil.copytree(os.path.join(REPO, "diplomjourney_amd", "csrc"),
                    os.path.join(d, "diplomjourney_amd", "csrc"))
    cs = os.path.join(d, "diplomjourney_amd", "csrc")
    st = lambda slot: STAMP.format(slot=slot)   # noqa: E731
    b0 = lambda q: f"if (blockIdx.x == 0 && threadIdx.x == 0) {st(B0_BASE + q)};"   # noqa: E731
    patch(os.path.join(cs, "mpc_kernels.h"), [
        ("                             __HIP_MEMORY_SCOPE_WORKGROUP);\n      }\n      if (early_on && q >= 192",
         "                             __HIP_MEMORY_SCOPE_WORKGROUP);\n"
         f"        if (blockIdx.x == 0 && q == 64) {STAMP.format(slot=B0_BASE + 18)};\n"
         "      }\n      if (early_on && q >= 192"),
        ("      __hip_atomic_store(&s_pose, ok ? 1 : 2, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);\n",
         "      __hip_atomic_store(&s_pose, ok ? 1 : 2, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);\n"
         f"      if (blockIdx.x == 0) {STAMP.format(slot=B0_BASE + 19)};\n"),
    ])
    patch(os.path.join(cs, "mpc_kernels.h"), [
        ("  __syncthreads();\n  key = s_key;\n", f"  __syncthreads();\n  {b0(16)}\n  key = s_key;\n"),
        ("  side_a();\n", f"  {b0(17)}\n  side_a();\n"),
    ])
    patch(os.path.join(cs, "mpc_kernels.h"), [
        ("struct Rec {\n", f"__device__ uint64_t g_tl[8 * {NB} + 32];\n\nstruct Rec {{\n"),
        ("  if (stage) s_head[threadIdx.x - 64] = head_word;\n",
         f"  {b0(1)}\n"
         "  if (stage) s_head[threadIdx.x - 64] = head_word;\n"),
        ("  wave_argmin(k, i);\n  // Each wave's best", f"  wave_argmin(k, i);\n  {b0(2)}\n  // Each wave's best"),
        ("  int wbest = 0;\n", f"  {b0(3)}\n  int wbest = 0;\n"),
        ("  if (KDEV && hook.H) {\n    const bool early = hook.publish_epoch && s_early;",
         f"  {b0(5)}\n  if (KDEV && hook.H) {{\n    const bool early = hook.publish_epoch && s_early;"),
        ("                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);\n      }\n    };\n",
         "                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);\n"
         f"        if (blockIdx.x == 0 && threadIdx.x == 192) {STAMP.format(slot=B0_BASE + 13)};\n"
         "      }\n    };\n"),
        ("                   early ? s_pub : nullptr, &bad);\n",
         f"                   early ? s_pub : nullptr, &bad);\n      {b0(7)}\n"),
        ("      *reinterpret_cast<EarlyPub*>(reinterpret_cast<uint64_t*>(hook.H) + kStoredWords) = E;\n",
         "      *reinterpret_cast<EarlyPub*>(reinterpret_cast<uint64_t*>(hook.H) + kStoredWords) = E;\n"
         f"      if (blockIdx.x == 0) {STAMP.format(slot=B0_BASE + 15)};\n"),
        ("    emit_winner_tail<INTEG, ROT>(K, n_steps, lds, out);\n  }\n}\n",
         f"    emit_winner_tail<INTEG, ROT>(K, n_steps, lds, out);\n    {b0(14)}\n  }}\n}}\n"),
        ("                 hook.chain_pub, hook.chain_pub_words, hook.publish_epoch, early, s_pub);\n",
         "                 hook.chain_pub, hook.chain_pub_words, hook.publish_epoch, early, s_pub);\n"
         f"    {b0(8)}\n"),
        ("  __syncthreads();\n  // Regular rotation-mode winner",
         f"  __syncthreads();\n  {b0(4)}\n  // Regular rotation-mode winner"),
    ])
    t = lambda q: f"if (threadIdx.x == 0) {STAMP.format(slot=f'8 * blockIdx.x + {q}')};"   # noqa: E731
    patch(os.path.join(cs, "mpc_episode.h"), [
        ("  block_argmin<true>(best_k, best_i);   // (indices < n_cand < 2^31)\n",
         f"  {t(4)}\n  block_argmin<true>(best_k, best_i);   // (indices < n_cand < 2^31)\n  {t(5)}\n"),
    ])
    patch(os.path.join(cs, "mpc_episode.h"), [
        # P2P block 0 (p2p_complete): candidate from the records, posted, the
        # world's gathered; published (advance_from_candidates' store_update)
        ("                           lc);\n  if (static_cast<int>(threadIdx.x) < world)",
         f"                           lc);\n  {b0(1)}\n  if (static_cast<int>(threadIdx.x) < world)"),
        ("  post_candidate(s_peers, s_rank, world, prev, slot, n_steps, lc);\n",
         f"  post_candidate(s_peers, s_rank, world, prev, slot, n_steps, lc);\n  {b0(2)}\n"),
        ("      wait_mailbox(S, mb, prev, slot, world, n_steps, s_err == 5u ? 0ull : kPeerWaitTicks);\n",
         "      wait_mailbox(S, mb, prev, slot, world, n_steps, s_err == 5u ? 0ull : kPeerWaitTicks);\n"
         f"  {b0(3)}\n"),
        ("               kPubWords, publish_epoch);\n  emit_winner_tail",
         f"               kPubWords, publish_epoch);\n  {b0(8)}\n  emit_winner_tail"),
        ("  EpisodeHead* S = &H;\n  S->steps_for_slowing -= 1;\n",
         f"  {b0(9)}\n  EpisodeHead* S = &H;\n  S->steps_for_slowing -= 1;\n"),
        ("  const double x_prev = S->x, y_prev = S->y;   // x_previous",
         f"  {b0(10)}\n  const double x_prev = S->x, y_prev = S->y;   // x_previous"),
        ("  if (early && (ended ||", f"  {b0(11)}\n  if (early && (ended ||"),
        ("  } else {\n    episode_prepare(c, *S);\n  }\n}\n",
         f"  }} else {{\n    episode_prepare(c, *S);\n  }}\n  {b0(12)}\n}}\n"),
        ("  L.status = status;\n  if (ended) {\n",
         f"  L.status = status;\n  {b0(6)}\n  if (ended) {{\n"),
        ("  if (blockIdx.x == 0) {\n    if (has_prev) {\n",
         f"  if (blockIdx.x == 0) {{\n    {t(0)}\n    if (has_prev) {{\n"),
        ("  constexpr int CPL = 2;\n  __shared__ __attribute__((aligned(16))) uint32_t s_w[kPubWords];\n",
         f"  {t(0)}\n  constexpr int CPL = 2;\n  __shared__ __attribute__((aligned(16))) uint32_t s_w[kPubWords];\n"),
        ("      if (threadIdx.x == 0) s_final = fin;\n    }\n    __syncthreads();\n",
         f"      if (threadIdx.x == 0) s_final = fin;\n    }}\n    __syncthreads();\n    {t(1)}\n"),
        ("S->chain_error = 1u;\n      }\n      __syncthreads();\n    }\n  };\n",
         f"S->chain_error = 1u;\n      }}\n      __syncthreads();\n    }}\n    {t(2)}\n  }};\n"),
        ("    else\n      part[blockIdx.x - 1] = Rec{best_k, best_i};\n  }\n}\n",
         "    else\n      part[blockIdx.x - 1] = Rec{best_k, best_i};\n"
         f"    asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");\n    {t(3)}\n  }}\n}}\n"),
    ])
    patch(os.path.join(cs, "mpc_rollout.hip"), [
        ("// ----------------------------- RCCL exchange",
         "extern \"C\" int mpc_debug_timeline(void* dst, size_t bytes) {\n"
         "  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(mpc::g_tl), bytes) == hipSuccess ? 0 : -1;\n"
         "}\n\n// ----------------------------- RCCL exchange"),
    ])
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-ldl", "-ffp-contract=off", "-I", os.path.join(d, "include"), "-o", VAR,
           os.path.join(cs, "mpc_rollout.hip")]
    r = subprocess.run(cmd, capture_output=True, text=True, cwd=d)
    shutil.rmtree(d)
    if r.returncode:
        raise SystemExit(r.stderr[-3000:])
    print(VAR)


B0_P2P = {1: "candidate", 2: "posted", 3: "gathered", 6: "advance", 8: "published"}


def run(n, ns, mode="chain"):
    sys.path.insert(0, REPO)
    from diplomjourney_amd import native
    native.LIB_PATH = VAR            # the timeline build (developer tool)
    import torch
    from diplomjourney_amd import math_model_tree as mmt
    from diplomjourney_amd import native
    from diplomjourney_amd.episode import DeviceEpisode
    from diplomjourney_amd.expansion import Expansion
    eng = Expansion("cuda:0")
    V = torch.tensor(mmt.vector_of_velocities(0.5), dtype=torch.float64, device="cuda")
    B = torch.tensor(mmt.vector_of_beta_angles(0.0), dtype=torch.float64, device="cuda")
    if mode == "tiled":   # the bench default's MPC_LAYOUT_TILED batches
        pool = [eng.sample_controls_tiled(V, B, n, ns, 0x5EED0000 + i) for i in range(8)]
    else:
        pool = [eng.sample_controls(V, B, n, ns, 0x5EED0000 + i) for i in range(8)]
    p2p = mode == "p2p"
    ep = DeviceEpisode(eng, n, ns, integrator="rect+cum", chain=True, log_capacity=8192,
                       exchange=p2p, p2p=p2p)
    L = native.lib()
    L.mpc_debug_timeline.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    nb = (n + 511) // 512 + 1
    buf = (ctypes.c_uint64 * (8 * NB + 32))()
    rows = []
    for rep in range(5):
        for i in range(300):
            ep.step(controls=pool[i % 8])
        torch.cuda.synchronize()
        assert L.mpc_debug_timeline(buf, ctypes.sizeof(buf)) == 0
        t = [buf[j] for j in range(8 * nb)]
        t0 = min(t[8 * b] for b in range(nb))
        us = lambda x: (x - t0) * 0.01   # noqa: E731
        b0 = {"entry": us(t[0])}
        names = B0_P2P if p2p else {q: name for q, name in enumerate(B0) if q}
        b0.update({name: us(buf[B0_BASE + q]) for q, name in names.items()})
        row = {"block0": b0}
        for q, name in enumerate(TILE):
            xs = sorted(us(t[8 * b + q]) for b in range(1, nb))
            row[name] = [xs[int(p * (len(xs) - 1))] for p in (0.1, 0.5, 0.9)] + [xs[-1]]
        rows.append(row)
    ep.flush()
    assert ep.chain_error() == 0
    print(f"chained step, {n} candidates, N = {ns}, {nb} blocks; us after the first block's entry")
    for r in rows:
        b0 = r["block0"]
        print("  block 0: " + "  ".join(f"{k} {v:5.2f}" for k, v in b0.items()))
        print("  tiles p10/p50/p90/max: " + "  ".join(
            f"{k} " + "/".join(f"{x:.2f}" for x in r[k]) for k in TILE))
    print("JSON " + json.dumps(rows))


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build()
    else:
        run(int(sys.argv[2]), int(sys.argv[3]), *(sys.argv[4:5]))
