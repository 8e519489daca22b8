"""In-step kernel durations from a rocprofv3 kernel trace of bench.py: the
longest run of alternating rollout / finalize dispatches (the graph-replayed
timed steps); medians of each kernel, of the gaps and of the step period.
    python tools/step_trace.py run_kernel_trace.csv [label]"""
import csv
import statistics as st
import sys


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    seq = [(r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").replace("mpc::", ""),
            int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
    roll = ("k_rollout_argmin", "k_rollout_argmin_stream")
    best, i = (0, 0), 0
    while i < len(seq):
        j = i
        while j + 1 < len(seq) and seq[j][0] in roll and seq[j + 1][0] == "k_finalize":
            j += 2
        if j - i > best[1] - best[0]:
            best = (i, j)
        i = j + 1 if j > i else i + 1
    chain = [x for x in seq if x[0] == "k_episode_chain"]
    if len(chain) > 2 * (best[1] - best[0]):
        # chained steps: one launch per step; the longest back-to-back run
        runs, cur = [], [chain[0]]
        for a, b in zip(chain, chain[1:]):
            if b[1] - a[2] < 5000:
                cur.append(b)
            else:
                runs.append(cur)
                cur = [b]
        runs.append(cur)
        run = max(runs, key=len)
        med = lambda v: round(st.median(v) / 1e3, 2)  # noqa: E731
        print({"label": sys.argv[2] if len(sys.argv) > 2 else "", "steps": len(run),
               "chain_us": med([e - s for n, s, e in run]),
               "gap_us": med([run[k + 1][1] - run[k][2] for k in range(len(run) - 1)]),
               "period_us": med([run[k + 1][1] - run[k][1] for k in range(len(run) - 1)])})
        return
    run = seq[best[0]:best[1]]
    med = lambda v: round(st.median(v) / 1e3, 2)  # noqa: E731
    out = {"label": sys.argv[2] if len(sys.argv) > 2 else "", "steps": len(run) // 2,
           "rollout_us": med([e - s for k, (n, s, e) in enumerate(run) if k % 2 == 0]),
           "finalize_us": med([e - s for k, (n, s, e) in enumerate(run) if k % 2 == 1]),
           "gap_rf_us": med([run[k + 1][1] - run[k][2] for k in range(0, len(run) - 1, 2)]),
           "gap_fr_us": med([run[k + 2][1] - run[k + 1][2] for k in range(0, len(run) - 2, 2)]),
           "period_us": med([run[k + 2][1] - run[k][1] for k in range(0, len(run) - 2, 2)])}
    print(out)


if __name__ == "__main__":
    main()
