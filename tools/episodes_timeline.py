"""Phase timeline of workload R's kernel (k_episodes_run: one block per robot
runs its episode's MPC steps back to back): a variant build with
s_memrealtime (100 MHz) stamps patched into a copy of the sources, summed per
phase over every call of block 0 (thread 0's view), then the mean per call.

    python tools/episodes_timeline.py build          # -> tools/tl_episodes.so (CPU)
    python tools/episodes_timeline.py run [R] [K]    # on the GPU box

Phases: grid (episode_grids + barrier), rollout (thread 0's own candidates),
argmin (block arg-min + barrier), re-roll (emit_winner), advance (thread 0:
episode_advance), log (barrier + log store)."""
import ctypes
import json
import os
import shutil
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VAR = os.path.join(REPO, "tools", "tl_episodes.so")   # git-ignored; delete after use
PH = ["grid", "rollout", "argmin", "re-roll", "advance", "log"]
NOW = "__builtin_amdgcn_s_memrealtime()"


def patch(path, edits):
    s = open(path).read()
    for anchor, new in edits:
        if s.count(anchor) != 1:
            raise SystemExit(f"{os.path.basename(path)}: anchor found {s.count(anchor)}x: {anchor!r}")
        s = s.replace(anchor, new)
    open(path, "w").write(s)


def build(src=None):
    d = tempfile.mkdtemp()
    shutil.copytree(os.path.join(REPO, "include"), os.path.join(d, "include"))
    shutil.copytree(os.path.join(REPO, "diplomjourney_amd", "csrc"),
                    os.path.join(d, "diplomjourney_amd", "csrc"))
    cs = os.path.join(d, "diplomjourney_amd", "csrc")
    mark = lambda q: f"if (threadIdx.x == 0) {{ const uint64_t tn = {NOW}; " \
                     f"tl_acc[{q}] += tn - tl_prev; tl_prev = tn; }}"   # noqa: E731
    patch(os.path.join(cs, "mpc_episodes.h"), [
        ("constexpr int32_t kEpEnded", "__device__ uint64_t g_tl_ep[8 * 65536];\n\nconstexpr int32_t kEpEnded"),
        ("  int64_t cands = 0;   // (thread 0)\n",
         "  int64_t cands = 0;   // (thread 0)\n  uint64_t tl_acc[6] = {0, 0, 0, 0, 0, 0};\n"
         f"  uint64_t tl_prev = {NOW};\n  int tl_n = 0;\n"),
        ("    if (s_stop) break;   // uniform\n",
         f"    if (s_stop) break;   // uniform\n    if (threadIdx.x == 0) {{ tl_prev = {NOW}; tl_n++; }}\n"),
        ("    const Consts K = uniform_consts(Hs->K);\n",
         f"    {mark(0)}\n    const Consts K = uniform_consts(Hs->K);\n"),
        ("    block_argmin<true>(best_k, best_i);\n    if (threadIdx.x == 0) {\n      s_bk = best_k;",
         f"    {mark(1)}\n    block_argmin<true>(best_k, best_i);\n    if (threadIdx.x == 0) {{\n      s_bk = best_k;"),
        ("    const uint64_t bk = s_bk;\n    const int64_t bi = s_bi;\n",
         f"    {mark(2)}\n    const uint64_t bk = s_bk;\n    const int64_t bi = s_bi;\n"),
        ("    if (threadIdx.x == 0) {   // (emit_winner, if it ran, ended with a barrier)\n",
         f"    {mark(3)}\n    if (threadIdx.x == 0) {{   // (emit_winner, if it ran, ended with a barrier)\n"),
        ("      s_calls += 1;\n    }\n",
         f"      s_calls += 1;\n    }}\n    {mark(4)}\n"),
        ("          [threadIdx.x] = reinterpret_cast<const uint64_t*>(&s_log)[threadIdx.x];\n  }\n",
         "          [threadIdx.x] = reinterpret_cast<const uint64_t*>(&s_log)[threadIdx.x];\n"
         f"    __syncthreads();\n    {mark(5)}\n  }}\n"
         "  if (threadIdx.x == 0) {\n"
         "    for (int q = 0; q < 6; ++q) g_tl_ep[8 * blockIdx.x + q] = tl_acc[q];\n"
         "    g_tl_ep[8 * blockIdx.x + 6] = tl_n;\n  }\n"),
    ])
    patch(os.path.join(cs, "mpc_rollout.hip"), [
        ("// ----------------------------- RCCL exchange",
         "extern \"C\" int mpc_debug_timeline(void* dst, size_t bytes) {\n"
         "  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(mpc::g_tl_ep), bytes) == hipSuccess ? 0 : -1;\n"
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


def run(R=1000, K=1000, integ="qk21"):
    sys.path.insert(0, REPO)
    from diplomjourney_amd import native
    native.LIB_PATH = VAR            # the timeline build (developer tool)
    import time
    import torch
    from diplomjourney_amd import run_math_model as rmm
    from diplomjourney_amd.episode import DeviceEpisodes, tree_episode_config
    from diplomjourney_amd.expansion import Expansion
    eng = Expansion("cuda:0")
    starts = rmm.draw_starts(R, seed=20261015)
    eps = DeviceEpisodes(eng, [tree_episode_config(s, K) for s in starts], 3, integ,
                         log_capacity=K)
    L = native.lib()
    L.mpc_debug_timeline.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    buf = (ctypes.c_uint64 * (8 * R))()
    for rep in range(3):
        eps.reset()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eps.run(K)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        calls, _, _ = eps.read_progress()
        assert L.mpc_debug_timeline(buf, ctypes.sizeof(buf)) == 0
        tl = [[buf[8 * r + q] for q in range(7)] for r in range(R)]
        longest = max(range(R), key=lambda r: tl[r][6])
        tot = [sum(tl[r][q] for r in range(R)) for q in range(7)]

        def fmt(row):
            n = max(1, row[6])
            per = {p: row[q] * 10.0 / n for q, p in enumerate(PH)}   # ns per call
            return per, "  ".join(f"{k} {v:.0f}" for k, v in per.items()) + \
                f"  total {sum(per.values()):.0f} ns/call over {n} calls"
        per, txt = fmt(tl[longest])
        print(f"run {dt * 1e3:.2f} ms ({dt / max(1, calls.max()) * 1e6:.2f} us/lockstep step)\n"
              f"  longest robot {longest}: {txt}\n  all robots: {fmt(tot)[1]}", flush=True)
    print("JSON " + json.dumps(per))


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build()
    else:
        run(*(int(a) for a in sys.argv[2:4]))
