"""Debug: the device full-tree episodes' first call vs the single-problem
full tree on the same problem (gold episode 0)."""
import json, os, sys
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
from diplomjourney_amd import run_math_model as rmm
from diplomjourney_amd.abi import MpcFulltreeEpisodeConfig, MpcFulltreeProblem
from diplomjourney_amd.episode import DeviceFtEpisodes
from diplomjourney_amd.expansion import fulltree_argmin, fulltree_result
g = json.load(open(os.path.join(REPO, "tests/golden/fulltree_reference.json")))
cfg = g["config"]
rmm.configure(cfg["delta_v"], cfg["delta_beta"])
eng, (vg, bg) = rmm._device()
for integ in ("qk21", "rect+rot"):
    for e in g["episodes"]:
        r = rmm._Robot((e["x_0"], e["y_0"], e["phi_0"], e["x_t"], e["y_t"]))
        c = MpcFulltreeEpisodeConfig(r.x_0, r.y_0, r.phi_0, r.x_t, r.y_t, r.atan_t, float(r.crit), 1, 0)
        ep = DeviceFtEpisodes(eng, [c], vg, bg, rmm.L, rmm.delta_t, rmm.eps, integ, log_capacity=4)
        ep.run(1)
        lg = ep.read_logs()[0]
        p = MpcFulltreeProblem(r.x, r.y, r.phi, r.x_t, r.y_t, r.x_0, r.y_0, r.atan_t, rmm.L, 0.05, 0.1)
        one = fulltree_result(fulltree_argmin(eng, p, vg, bg, float(r.crit), integ))
        print(integ, "device-episode leaf", int(lg["index"][0]), "crit", float(lg["cost"][0]),
              "| single", one.leaf, one.cost, "| ret", [float(lg[k][0]) for k in ("x", "y", "phi", "v", "beta")],
              one.trajectory()[0])
