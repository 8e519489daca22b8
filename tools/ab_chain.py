"""Same-box A/B of library builds at config C: for each library (env
tools/with_lib.py <path>, one child process per measurement, interleaved
for R rounds) the chained launch and the plain streaming kernel, 300 warm +
200 timed back-to-back launches between HIP events over 8 resident batches.
    python tools/ab_chain.py ROUNDS LIB [LIB ...]      (LIB "-" = in-tree build)"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    sys.path.insert(0, REPO)
    import torch
    from diplomjourney_amd import math_model_tree as mmt
    from diplomjourney_amd.episode import DeviceEpisode
    from diplomjourney_amd.expansion import Expansion
    n = int(os.environ.get("AB_N", "1000000"))
    ns = int(os.environ.get("AB_NS", "10"))
    eng = Expansion("cuda:0")
    V = torch.tensor(mmt.vector_of_velocities(0.5), dtype=torch.float64, device="cuda")
    B = torch.tensor(mmt.vector_of_beta_angles(0.0), dtype=torch.float64, device="cuda")
    pool = [eng.sample_controls(V, B, n, ns, 0x5EED0000 + i) for i in range(8)]
    if os.environ.get("AB_PAD"):
        # v and beta of a batch in ONE allocation with a tile of padding after
        # them, so a variant reading tile-contiguous blocks stays in bounds
        padded = []
        for v, b in pool:
            buf = torch.empty(2 * ns * n + ns * 1024, dtype=torch.float64, device="cuda")
            buf[:ns * n].copy_(v.reshape(-1))
            buf[ns * n:2 * ns * n].copy_(b.reshape(-1))
            buf[2 * ns * n:].fill_(0.25)
            padded.append((buf[:ns * n].view(ns, n), buf[ns * n:2 * ns * n].view(ns, n), buf))
        pool = [(v, b) for v, b, _ in padded]
        keep = padded   # noqa: F841 (holds the buffers)
    tpool = pool
    if os.environ.get("AB_TILED"):   # the bench default's MPC_LAYOUT_TILED batches
        tpool = [eng.sample_controls_tiled(V, B, n, ns, 0x5EED0000 + i) for i in range(8)]
    ep = DeviceEpisode(eng, n, ns, integrator="rect+cum", chain=True, log_capacity=8192)
    out = {}
    for name, fn in (("chain", lambda i: ep.step(controls=tpool[i % 8])),
                     ("stream", lambda i: (setattr(ep, "cur", pool[i % 8]), ep.partials()))):
        for i in range(300):
            fn(i)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(200):
            fn(i + 3)
        e1.record()
        torch.cuda.synchronize()
        out[name] = e0.elapsed_time(e1) / 200 * 1e3
        ep.flush()
    print("AB " + json.dumps(out), flush=True)


def main():
    if sys.argv[1] == "--child":
        return child()
    rounds, libs = int(sys.argv[1]), sys.argv[2:]
    res = {lib: [] for lib in libs}
    for _ in range(rounds):
        for lib in libs:
            env = dict(os.environ)
            cmd = [sys.executable, os.path.abspath(__file__), "--child"]
            if lib != "-":
                cmd = [sys.executable, os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                    "with_lib.py"), os.path.abspath(lib)] + cmd[1:]
            r = subprocess.run(cmd, env=env,
                               capture_output=True, text=True, timeout=300)
            line = [ln for ln in r.stdout.splitlines() if ln.startswith("AB ")]
            if r.returncode != 0 or not line:
                print(lib, "failed", r.stderr[-800:], flush=True)
                return 1
            res[lib].append(json.loads(line[0][3:]))
    for lib, xs in res.items():
        ch = [x["chain"] for x in xs]
        stv = [x["stream"] for x in xs]
        print(f"{lib:32s} chain " + " ".join(f"{x:6.2f}" for x in ch) + f"  min {min(ch):6.2f}"
              f" | stream " + " ".join(f"{x:6.2f}" for x in stv) + f"  min {min(stv):6.2f} us",
              flush=True)


if __name__ == "__main__":
    sys.exit(main())
