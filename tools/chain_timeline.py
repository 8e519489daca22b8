"""Per-block timeline of one chained launch (config C by default), from a
debug build with -DMPC_CHAIN_TIMELINE:

  tools/build_variant.sh tl -DMPC_CHAIN_TIMELINE
  DIPLOMJOURNEY_MPC_LIB=tools/var_tl.so python tools/chain_timeline.py [n] [ns]

Prints (µs from the launch's first block entry): when blocks enter (dispatch
ramp), the first-DMA/constants wait (pre0), the loop, the final-constants wait,
the record, the tail (how many blocks are still streaming over time), and a
per-XCC summary.  Timing probe only; results are not checked."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from diplomjourney_amd import math_model_tree as mmt  # noqa: E402
from diplomjourney_amd import native  # noqa: E402
from diplomjourney_amd.episode import DeviceEpisode  # noqa: E402
from diplomjourney_amd.expansion import Expansion  # noqa: E402

TL_BLOCKS = 8192


def pct(a, q):
    return float(np.percentile(a, q))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    ns = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    eng = Expansion("cuda:0")
    V = torch.tensor(mmt.vector_of_velocities(0.5), dtype=torch.float64, device="cuda")
    B = torch.tensor(mmt.vector_of_beta_angles(0.0), dtype=torch.float64, device="cuda")
    pool = [eng.sample_controls(V, B, n, ns, 0x5EED0000 + i) for i in range(8)]
    ep = DeviceEpisode(eng, n, ns, integrator="rect+cum", chain=True, log_capacity=8192)
    lib = native.lib()
    lib.mpc_debug_chain_timeline.argtypes = [ctypes.c_void_p]
    buf = np.zeros((TL_BLOCKS, 6), dtype=np.uint64)
    for i in range(400):                      # warm clocks; steady back-to-back launches
        ep.step(controls=pool[i % 8])
    torch.cuda.synchronize()
    reports = []
    for rep in range(3):
        for i in range(50):
            ep.step(controls=pool[i % 8])     # the timeline is the last launch's
        native.check(lib.mpc_debug_chain_timeline(buf.ctypes.data), "timeline")
        # this launch's blocks: entered at most 10 µs before block 0 (the
        # buffer keeps older launches' rows beyond a shorter grid)
        ent = buf[:, 0].astype(np.int64)
        grid = int(np.nonzero(ent >= ent[0] - 1000)[0].max()) + 1
        t = buf[:grid, :5].astype(np.int64)
        xcc = buf[:grid, 5].astype(np.int64)
        t0 = t[:, 0].min()
        us = (t - t0) / 100.0                 # 100 MHz ticks -> µs
        tiles = us[1:]
        entry, pre, lend, wdone, rec = (tiles[:, k] for k in range(5))
        end = rec.max()
        reports.append(end)
        print(f"--- launch {rep}: {grid} blocks, first entry -> last record {end:.2f} us")
        print(f"block 0: entry {us[0, 0]:.2f}, published {us[0, 4]:.2f}")
        print("entry      p0 %.2f p10 %.2f p50 %.2f p90 %.2f max %.2f" % tuple(
            pct(entry, q) for q in (0, 10, 50, 90, 100)))
        for name, a in (("pre0 wait", pre - entry), ("loop", lend - pre),
                        ("final wait", wdone - lend), ("record", rec - wdone),
                        ("lifetime", rec - entry)):
            print("%-10s p10 %.2f p50 %.2f p90 %.2f max %.2f" % (
                (name,) + tuple(pct(a, q) for q in (10, 50, 90, 100))))
        # how many blocks stream (entered, no record yet) over time
        grid_t = np.arange(0.0, end + 0.5, 1.0)
        live = [int(((entry <= x) & (rec > x)).sum()) for x in grid_t]
        print("live blocks per µs: " + " ".join(str(v) for v in live))
        first_round = entry < pct(entry, 50)
        print(f"late-entry blocks (entered after {pct(entry, 60):.2f} us): lifetime p50 "
              f"{pct((rec - entry)[entry > pct(entry, 60)], 50):.2f} vs early "
              f"{pct((rec - entry)[first_round], 50):.2f}")
        for x in range(8):
            m = xcc[1:] == x
            if m.any():
                print(f"xcc {x}: {int(m.sum())} blocks, last record {rec[m].max():.2f}, "
                      f"mean lifetime {(rec - entry)[m].mean():.2f}")
    ep.flush()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
