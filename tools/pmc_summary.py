"""Summarise tools/pmc.sh counter passes for the rollout kernel into a JSON
file bench.py reads for roofline.traffic (--traffic-json).

    python tools/pmc_summary.py gpurun_out/<tag> out.json [algorithmic_bytes] [kernel] [label] [layout] [sum]

kernel: a substring of the rocprof kernel name (e.g. "k_episode_chain<1, 2, 3"
for the exchange form); label: the name written to the summary's "kernel"
field, the key bench.py matches (default: kernel).  sum: the counters of EVERY
matching dispatch of a pass added up as one "launch" (a run of several
kernels, e.g. workload G's lockstep calls: three launches per call).

HBM bytes per launch = 2 x FETCH_SIZE (KB x 1024) + WRITE_SIZE: on gfx950
FETCH_SIZE counts half the bytes of a 16-B-per-lane streaming read and
WRITE_SIZE is exact for 16-B stores (MI355X_MICROARCH.md, HBM section)."""
import collections
import csv
import glob
import json
import os
import sys


def main():
    root, out = sys.argv[1], sys.argv[2]
    algo = float(sys.argv[3]) if len(sys.argv) > 3 else 160e6   # 16 B x N x C of the runs
    kernel = sys.argv[4] if len(sys.argv) > 4 else "k_rollout_argmin_stream"
    label = sys.argv[5] if len(sys.argv) > 5 else kernel
    layout = sys.argv[6] if len(sys.argv) > 6 else "soa"   # the controls' layout of the runs
    whole_run = len(sys.argv) > 7 and sys.argv[7] == "sum"
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in sorted(glob.glob(os.path.join(root, "pmc*", "p_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            if kernel not in r["Kernel_Name"]:
                continue
            key = (f,) if whole_run else (f, r["Dispatch_Id"])
            per[r["Counter_Name"]][key] += float(r["Counter_Value"])
    med = {}
    for name, d in per.items():
        xs = sorted(d.values())
        med[name] = xs[len(xs) // 2]
    fetch_b = med.get("FETCH_SIZE", 0.0) * 1024.0
    write_b = med.get("WRITE_SIZE", 0.0) * 1024.0
    f64 = None
    if "SQ_INSTS_VALU_FMA_F64" in med:
        # fp64 operations per launch, 64 lanes per wave-instruction (an upper
        # bound: inactive lanes count); FMA = 2
        f64 = 64.0 * (2 * med["SQ_INSTS_VALU_FMA_F64"] + med.get("SQ_INSTS_VALU_ADD_F64", 0)
                      + med.get("SQ_INSTS_VALU_MUL_F64", 0) + med.get("SQ_INSTS_VALU_TRANS_F64", 0))
    res = {
        "kernel": label,
        "layout": layout,
        "kernel_name_filter": kernel,
        "fp64_ops_per_launch": f64,
        "hbm_bytes_per_launch": 2.0 * fetch_b + write_b,
        "algorithmic_bytes_per_launch": algo,
        "fetch_size_bytes_raw": fetch_b, "write_size_bytes": write_b,
        "correction": "2 x FETCH_SIZE (gfx950 16-B streaming reads) + WRITE_SIZE",
        "counters_median_per_launch": med,
        "source": os.path.relpath(root),
    }
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "counters_median_per_launch"}))


if __name__ == "__main__":
    main()
