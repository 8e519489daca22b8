"""Shader clock (s_memtime / s_memrealtime) across K=20 graph replays of the
chained steps, each replay after a sync (the driver's timed region) — is the
per-replay spread a clock effect?   python tools/micro/clock_replay.py [K]"""
import ctypes
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)


def main():
    import torch
    from diplomjourney_amd import math_model_tree as mmt
    from diplomjourney_amd.episode import DeviceEpisode
    from diplomjourney_amd.expansion import Expansion
    lib = ctypes.CDLL(os.path.join(REPO, "tools/micro/libclock.so"))
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    eng = Expansion("cuda:0")
    V = torch.tensor(mmt.vector_of_velocities(0.5), dtype=torch.float64, device="cuda")
    B = torch.tensor(mmt.vector_of_beta_angles(0.0), dtype=torch.float64, device="cuda")
    n, ns = 1_000_000, 10
    pool = [eng.sample_controls_tiled(V, B, n, ns, 0x5EED0000 + i) for i in range(K)]
    ep = DeviceEpisode(eng, n, ns, integrator="rect+cum", chain=True, log_capacity=8192)
    for i in range(5):
        ep.step(controls=pool[i])
    ep.flush()
    buf = torch.zeros(4, dtype=torch.int64, device="cuda")

    def stamp(i):
        s = torch.cuda.current_stream().cuda_stream
        assert lib.clock_stamp(ctypes.c_void_p(buf.data_ptr()), i, ctypes.c_void_p(s)) == 0

    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        stamp(0)
        for i in range(K):
            ep.step(controls=pool[i])
        ep.flush()
        stamp(1)
    rows = []
    for rep in range(40):
        if rep % 10 == 0:               # the bench's warm phase: ~300 steps back to back
            for _ in range(max(1, 300 // K)):
                g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        host = (time.perf_counter() - t0) * 1e6 / K
        t0c, r0, t1c, r1 = [int(x) for x in buf.tolist()]
        dev = (r1 - r0) * 10.0 / 1000 / K            # us per step (100 MHz)
        ghz = (t1c - t0c) / ((r1 - r0) * 10.0)       # memtime ticks per ns
        rows.append((host, dev, ghz))
        print(f"rep {rep:2d} host {host:6.2f} us/step  device {dev:6.2f} us/step  "
              f"memtime/ns {ghz:6.3f}", flush=True)
    rows.sort()
    print("fastest 5:", [f"{h:.1f}/{c:.3f}" for h, _, c in rows[:5]])
    print("slowest 5:", [f"{h:.1f}/{c:.3f}" for h, _, c in rows[-5:]])
    ep.flush()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
