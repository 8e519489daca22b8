"""Per-unit timeline of the persistent run (debug variant -DMPC_RUN_STATS):
per step, when its units started / ended streaming, were kept and
completed, against the selection (published head) times.
    DIPLOMJOURNEY_MPC_LIB=tools/var_stats.so python tools/unit_timeline.py [n] [ns] [K]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from diplomjourney_amd import math_model_tree as mmt, native  # noqa: E402
from diplomjourney_amd.episode import DeviceEpisode  # noqa: E402
from diplomjourney_amd.expansion import Expansion  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    ns = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 100
    eng = Expansion("cuda:0")
    L = native.lib()
    ut = L.mpc_debug_run_unit_times
    ut.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    V = torch.tensor(mmt.vector_of_velocities(0.5), dtype=torch.float64, device="cuda")
    B = torch.tensor(mmt.vector_of_beta_angles(0.0), dtype=torch.float64, device="cuda")
    pool = [eng.sample_controls(V, B, n, ns, 0x5EED0000 + i) for i in range(min(K, 40))]
    batches = [pool[i % len(pool)] for i in range(K)]
    ep = DeviceEpisode(eng, n, ns, integrator="rect+cum", log_capacity=8192)
    ep.run(batches[:10])
    ep._ptr_table(batches)
    clock = torch.zeros(K, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    ep.run(batches, clock=clock)
    torch.cuda.synchronize()
    T = -(-n // 512)
    nu = min(T * K, 1 << 20)
    buf = np.zeros(nu * 8, dtype=np.uint64)
    ut(buf.ctypes.data, nu)
    raw = buf.reshape(nu, 8).astype(np.float64)
    t = raw[:, [0, 1, 2, 3]]   # stream start, stream end, kept, record written
    pub = clock.cpu().numpy().astype(np.float64)   # step j's successor head published
    t0 = t[:T, 0].min()
    t = (t - t0) * 1e-2
    pub = (pub - t0) * 1e-2
    steps = min(K, nu // T)
    print(f"n={n} ns={ns} K={K} T={T}; us from the first unit start")
    print("step: start[min,med,max]  end[min,med,max]  complete[max]  P_j(head j published)  "
          "kept->record med  end-start med")
    for j in list(range(0, 4)) + list(range(steps // 2, steps // 2 + 6)):
        u = t[j * T:(j + 1) * T]
        pj = pub[j - 1] if j > 0 else 0.0
        print(f"{j:4d}: {u[:,0].min():8.1f} {np.median(u[:,0]):8.1f} {u[:,0].max():8.1f} | "
              f"{u[:,1].min():8.1f} {np.median(u[:,1]):8.1f} {u[:,1].max():8.1f} | {u[:,3].max():8.1f} | "
              f"{pj:8.1f} | {np.median(u[:,3]-u[:,2]):6.1f} {np.median(u[:,1]-u[:,0]):6.1f}")
    mid = slice((steps // 4) * T, (3 * steps // 4) * T)
    m = t[mid]
    print("medians over the middle half: stream (end-start)", np.median(m[:, 1] - m[:, 0]),
          "| full-hand wait (kept-end)", np.median(m[:, 2] - m[:, 1]),
          "| kept->record", np.median(m[:, 3] - m[:, 2]))
    per = np.diff(pub[steps // 4: 3 * steps // 4])
    print("period median", np.median(per), "chain_error", ep.chain_error())
    # units whose head was out when they were kept
    jj = np.arange(nu)[mid] // T
    pj = np.array([pub[j - 1] if j > 0 else -1e9 for j in jj])
    known = m[:, 2] >= pj
    print("units kept with their head already out:", known.mean(),
          "| their kept -> record", np.median((m[:, 3] - m[:, 2])[known]),
          "| others: head out -> record", np.median((m[:, 3] - pj)[~known]))
    # per block: busy (streaming) vs the gaps between its units
    blk = buf.reshape(nu, 8)[:, 7].astype(np.int64)[mid]
    lo, hi = m[:, 0].min(), m[:, 1].max()
    gaps_park, gaps_next, busy, nblk = [], [], 0.0, 0
    for b in np.unique(blk):
        r = m[blk == b]
        r = r[np.argsort(r[:, 0])]
        busy += (r[:, 1] - r[:, 0]).sum()
        nblk += 1
        gaps_park += list(r[:, 2] - r[:, 1])
        gaps_next += list(r[1:, 0] - r[:-1, 2])
    span = hi - lo
    print(f"blocks seen {nblk}; streaming fraction {busy / (nblk * span):.2f} of {span:.0f} us")
    st = m[:, 1] - m[:, 0]
    print("stream time per unit: p10 %.2f p50 %.2f p90 %.2f p99 %.2f max %.2f" %
          tuple(np.percentile(st, [10, 50, 90, 99, 100])))
    per_blk = np.array([st[blk == b].mean() for b in np.unique(blk)])
    print("per-block mean stream time: p10 %.2f p50 %.2f p90 %.2f max %.2f" %
          tuple(np.percentile(per_blk, [10, 50, 90, 100])))
    # lag: how far each block's unit starts trail the step's first start
    jj_mid = np.arange(nu)[mid] // T
    first = {j: m[jj_mid == j, 0].min() for j in np.unique(jj_mid)}
    lag = m[:, 0] - np.array([first[j] for j in jj_mid])
    lag_blk = np.array([lag[blk == b].mean() for b in np.unique(blk)])
    print("per-block mean start lag behind the step's first start: p10 %.1f p50 %.1f p90 %.1f max %.1f"
          % tuple(np.percentile(lag_blk, [10, 50, 90, 100])))
    for name, g in (("end->kept", gaps_park), ("kept->next start", gaps_next)):
        g = np.array(g)
        print(f"  {name}: p50 {np.percentile(g, 50):.2f} p90 {np.percentile(g, 90):.2f} "
              f"p99 {np.percentile(g, 99):.2f} mean {g.mean():.2f} us")


if __name__ == "__main__":
    main()
