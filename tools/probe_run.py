"""Phase counters of the persistent run (debug variant built with
tools/build_variant.sh stats -DMPC_RUN_STATS, loaded via
DIPLOMJOURNEY_MPC_LIB=tools/var_stats.so).
    python tools/probe_run.py [n_cand] [n_steps] [K]"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from diplomjourney_amd import math_model_tree as mmt, native  # noqa: E402
from diplomjourney_amd.episode import DeviceEpisode  # noqa: E402
from diplomjourney_amd.expansion import Expansion  # noqa: E402

NAMES = {8: "selector ticks sweep", 9: "selector ticks emit", 10: "selector ticks advance+pub",
         11: "sweep polls", 31: "registered blocks (summed over launches)"}


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    ns = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    eng = Expansion("cuda:0")
    L = native.lib()
    fn = L.mpc_debug_run_stats
    fn.argtypes = [ctypes.c_void_p]
    ep = DeviceEpisode(eng, n, ns, integrator="rect+cum", log_capacity=8192)
    V = torch.tensor(mmt.vector_of_velocities(0.5), dtype=torch.float64, device="cuda")
    B = torch.tensor(mmt.vector_of_beta_angles(0.0), dtype=torch.float64, device="cuda")
    pool = [eng.sample_controls(V, B, n, ns, 0x5EED0000 + i) for i in range(min(K, 60))]
    batches = [pool[i % len(pool)] for i in range(K)]
    ep.run(batches[:20])
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * 32)()
    fn(buf)
    tl_fn = L.mpc_debug_run_timeline
    tl_fn.argtypes = [ctypes.c_void_p]
    tl = (ctypes.c_ulonglong * 2560)()
    tl_fn(tl)
    ep._ptr_table(batches)
    clock = torch.zeros(K, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ep.run(batches, clock=clock)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    fn(buf)
    st = list(buf)
    c = clock.cpu().tolist()
    per = [(b - a) * 10e-3 for a, b in zip(c, c[1:])]
    per.sort()
    print(f"n={n} ns={ns} K={K}: {dt / K * 1e6:.1f} us/step wall, period p50 {per[len(per) // 2]:.1f} us")
    u = 1
    for i, name in NAMES.items():
        extra = ""
        if "ticks" in name and "selector" not in name:
            extra = f"  -> {st[i] / u * 10e-3:.2f} us per wait"
        if "selector" in name:
            extra = f"  -> {st[i] / K * 10e-3:.2f} us per step"
        print(f"  {name:32s} {st[i]}{extra}")
    tl_fn(tl)
    rows = [tl[5 * j:5 * j + 5] for j in range(min(K, 512))]
    t0 = rows[0][0]
    print("timeline (us from step 0's first stream start): first-start last-end last-complete sweep-done published")
    for j in list(range(0, 6)) + list(range(K // 2, K // 2 + 6)):
        r = rows[j]
        print(f"  step {j:4d}: " + " ".join(f"{(x - t0) * 1e-2:9.1f}" for x in r))
    import statistics as stt
    d = lambda a, b: [(rows[j][a] - rows[j][b]) * 1e-2 for j in range(10, K - 2)]  # noqa: E731
    print("median us: last-end - first-start", stt.median(d(1, 0)),
          "| complete - last-end", stt.median(d(2, 1)),
          "| sweep - complete", stt.median(d(3, 2)), "| publish - sweep", stt.median(d(4, 3)))
    nxt = [(rows[j + 1][0] - rows[j][0]) * 1e-2 for j in range(10, K - 2)]
    pub_to_lastend = [(rows[j + 1][1] - rows[j][4]) * 1e-2 for j in range(10, K - 2)]
    print("median us: first-start(j+1) - first-start(j)", stt.median(nxt),
          "| last-end(j+1) - published(j)", stt.median(pub_to_lastend))
    print("chain_error", ep.chain_error())


if __name__ == "__main__":
    main()
