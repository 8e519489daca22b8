"""Host-timed cost of HIP timing events around a graph replay: the bench's
timed region (one replay of the K chained steps + flush between syncs) with
and without a timing event recorded before and after the replay, and with the
events captured inside the graph, interleaved.   python tools/micro/event_overhead.py [K]"""
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)


def main():
    import torch
    from diplomjourney_amd import math_model_tree as mmt
    from diplomjourney_amd.episode import DeviceEpisode
    from diplomjourney_amd.expansion import Expansion
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
    torch.cuda.synchronize()
    Ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(K):
            ep.step(controls=pool[i])
        ep.flush()
    gi = torch.cuda.CUDAGraph()
    ei0, ei1 = Ev(), Ev()
    with torch.cuda.graph(gi):
        ei0.record()
        for i in range(K):
            ep.step(controls=pool[i])
        ep.flush()
        ei1.record()
    for _ in range(15):
        g.replay()
    torch.cuda.synchronize()
    res = {"plain": [], "events": [], "in_graph": []}
    dev = {"events": [], "in_graph": []}
    for _ in range(int(os.environ.get('EVO_N', '12'))):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        res["plain"].append((time.perf_counter() - t0) * 1e6 / K)
        e0, e1 = Ev(), Ev()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        res["events"].append((time.perf_counter() - t0) * 1e6 / K)
        dev["events"].append(e0.elapsed_time(e1) * 1e3 / K)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        gi.replay()
        torch.cuda.synchronize()
        res["in_graph"].append((time.perf_counter() - t0) * 1e6 / K)
        try:
            dev["in_graph"].append(ei0.elapsed_time(ei1) * 1e3 / K)
        except Exception as e:   # noqa: BLE001
            dev["in_graph"].append(float("nan"))
    # the bench's sequence: ~15 warm replays, ONE sync (the host waits ~10 ms),
    # then the timed replay — with and without a host spin before it
    for mode in ("bench", "bench+spin", "bench", "bench+spin", "bench", "bench+spin",
                 "bench", "bench+spin"):
        for _ in range(15):
            g.replay()
        torch.cuda.synchronize()
        if mode.endswith("spin"):
            t_end = time.perf_counter() + 0.003
            while time.perf_counter() < t_end:
                pass
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.replay()
        t_sub = time.perf_counter()
        torch.cuda.synchronize()
        res.setdefault(mode, []).append((time.perf_counter() - t0) * 1e6 / K)
        res.setdefault(mode + " submit", []).append((t_sub - t0) * 1e6 / K)
    print("plain sorted:", " ".join(f"{x:.1f}" for x in sorted(res["plain"])))
    for mode in ("bench", "bench+spin", "bench submit", "bench+spin submit"):
        print(mode, " ".join(f"{x:.1f}" for x in res.pop(mode)))
    for k, v in res.items():
        print(f"{k:9s} host us/step median {statistics.median(v):7.2f}  min {min(v):7.2f}"
              + (f"  | device us/step median {statistics.median(dev[k]):7.2f}" if k in dev else ""))
    ep.flush()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
