"""Per-kernel durations and the gaps between consecutive dispatches from a
rocprofv3 kernel trace (CSV), over the last N dispatches of a kernel pattern's
steady state.  Shows where an MPC step's time goes between launches.
    python tools/trace_gaps.py <kernel_trace.csv> [last_n=600]"""
import collections
import csv
import re
import sys


def short(name):
    m = re.search(r"(k_[a-z_]+|ncclDevKernel\w*|[A-Za-z_]*Kernel\w*)", name)
    return m.group(1) if m else name[:40]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 600
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[-n:]
    dur = collections.defaultdict(list)
    gaps = collections.defaultdict(list)
    prev = None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        k = short(r["Kernel_Name"])
        dur[k].append((e - s) / 1e3)
        if prev is not None:
            gaps[(prev[0], k)].append((s - prev[1]) / 1e3)
        prev = (k, e)
    med = lambda xs: sorted(xs)[len(xs) // 2]
    print(f"last {len(rows)} dispatches, span {(int(rows[-1]['End_Timestamp']) - int(rows[0]['Start_Timestamp'])) / 1e3:.1f} us")
    for k, xs in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        print(f"  {k:40s} n={len(xs):5d} median {med(xs):8.2f} us  mean {sum(xs) / len(xs):8.2f} us")
    for (a, b), xs in sorted(gaps.items(), key=lambda kv: -len(kv[1])):
        print(f"  gap {a} -> {b}: n={len(xs)} median {med(xs):.2f} us  mean {sum(xs) / len(xs):.2f} us")


if __name__ == "__main__":
    main()
