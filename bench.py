#!/usr/bin/env python3
"""Benchmark: candidate N-step rollouts/s + MPC-step p50 latency (BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload C]
    torchrun --nproc-per-node N bench.py --gpus N ...      (one rank per GPU)

Workloads:
  C (default)  N=10 horizon, 1e6 candidates per GPU, moving-target episode
               (reference operator schedule); by default each step's candidate
               batch is already resident in HBM (--inputs resident; the grid
               regenerated per step around the chosen control and sampled on
               device is --inputs sampled / generated, both also reported in
               the line); weak scaling: 1e6 x G candidates over G GPUs
  B            N=3, 1e5 candidates per GPU, same episode machinery
  D            N=12, 1.25e6 candidates per GPU (1e7 over 8), one exchange/step
  E            1024 robots x 1e4 candidates, N=8, batched per-robot arg-min,
               robots sharded over GPUs (128 per GPU at 8), no exchange

A "step" is one MPC step of the device-resident episode (state in HBM, no
host synchronisation inside the loop):
  --inputs resident (default)  the step's candidate batch is already in HBM
      (a distinct synthetic batch per step, generated before the timed
      region).  Default (--integrator rect+cum): ONE chained launch per step,
      the rollout/arg-min of step k + the completion of step k-1 (winner
      re-roll + episode update: finishing logic, operator events, next step's
      problem).  --no-chain or another integrator: rollout
      kernel -> finalize kernel.  --step-form run: the K steps as ONE
      persistent launch per 64 steps (mpc_episode_run; bitwise the chained
      steps, slower on MI355X: DESIGN.md §6c "Persistent run")
  --inputs sampled  the device sampler first regenerates the candidates on the
      grid around the episode's current control (the reference's per-step
      grid), then the same two kernels
On G > 1 GPUs the per-rank winners are exchanged with one RCCL all_gather
before the episode update.  `value` is timed over K steps replayed from a HIP
graph (the RCCL all_gather captured with the kernels on G > 1; gloo
rehearsals launch eagerly); p50/p90 come from a separate
eager pass with HIP events; `other_inputs` repeats the run with the other
input mode.  --host-loop runs the host-driven episode instead.

Rank 0 prints ONE JSON line.  `roofline` is for the dominant kernel (the
chained k_episode_chain by default, k_rollout_argmin_stream for two-launch
steps): algorithmic bytes 16 B per candidate-step (fp64 v and beta read once)
/ its average duration, from HIP events around a graph replay of 200
back-to-back launches on the episode's stream and controls (graph_timed);
with chained steps `roofline_rollout_only` adds the same controls through the
rollout kernel alone.
`cpu_baseline` is the reference-structured Python port (scipy quad) on this
host's cores, rank 0 at N=1 only, on a bounded sample of the same candidates;
it runs before the GPU is initialised (it forks worker processes).
"""
import argparse
import gc
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "candidate N-step rollouts/sec + MPC-step p50 latency, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
D_TOTAL = 10_000_000    # config D's candidate total (BASELINE.json configs[3])

WORKLOADS = {
    "A": dict(n_steps=3, per_gpu=None,
              desc="config A: the reference scenario (math_model_tree.py:736-738, 349 "
                   "predictive_control calls, N=3, the acceleration-limited grid <= 451 "
                   "candidates) through the drop-in predictive_control"),
    "B": dict(n_steps=3, per_gpu=100_000, desc="config B: N=3, 1e5 candidates/GPU, episode"),
    "C": dict(n_steps=10, per_gpu=1_000_000,
              desc="config C: N=10, 1e6 candidates/GPU, moving-target episode"),
    "D": dict(n_steps=12, per_gpu=1_250_000,
              desc="config D: N=12, 1.25e6 candidates/GPU (1e7 at 8 GPUs), RCCL exchange"),
    "E": dict(n_steps=8, per_gpu=None, robots=1024, cand=10_000,
              desc="config E: 1024 robots x 1e4 candidates, N=8, batched per-robot arg-min"),
    "F": dict(n_steps=3, per_gpu=None,
              desc="full tree of run_math_model.py (SURVEY 8f 3): S1 = 11 x 41 controls, "
                   "S1^3 = 9.17e7 leaves per MPC step, heading-term criterion, never-reset "
                   "incumbent; episode of the run_math_model drop-in"),
}
WORKLOADS["R"] = dict(n_steps=3, per_gpu=None, robots=1000,
                      desc="run_math_model.py's 1000-episode loop (:231-280) over the tree "
                           "expansion of math_model_tree.py (acceleration-limited grid <= 451 "
                           "candidates, N=3): one robot per episode, device-resident, one "
                           "block per robot (mpc_episodes_run)")
WORKLOADS["G"] = dict(n_steps=3, per_gpu=None, robots=1000,
                      desc="run_math_model.py's 1000 episodes (SURVEY 8f 4): one robot per "
                           "episode, device-resident lockstep over the robots still running "
                           "(each call's leaves spread over the whole GPU), S1 = 5 x 13 "
                           "controls (274,625 leaves per robot-step)")
FP64_VECTOR_PEAK_TFLOPS = 78.6   # MI355X spec (2 x 32 lanes x 2 flops/clk/SIMD at 2.4 GHz / 2)
# fp64 operations per full-tree leaf (csrc/mpc_fulltree.h, one layer step + criterion), as
# written (an fma = 2): rect+rot 29 (heading add 1, rotation 6, two fused position updates 4,
# criterion 18 with its per-problem terms folded, ft_crit); qk21 adds 2 x 22 per leaf (two
# 21-node Kronrod sums + scaling).
FT_FLOPS_PER_LEAF = {"rect+rot": 29, "rect": 29, "qk21+rot": 73, "qk21": 73}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks, one per GPU; without a launcher (WORLD_SIZE unset) N > 1 "
                         "starts the N rank processes itself; under a launcher it must "
                         "equal WORLD_SIZE")
    ap.add_argument("--print-ranks", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (default 500 for the ~40 us expansion workloads, so the "
                         "fixed graph-launch + sync cost (~0.2 ms) is amortised; 50 for F/G)")
    ap.add_argument("--warmup", type=int, default=None,
                    help="untimed steps first (default 20; 1 scenario run for workload A)")
    ap.add_argument("--ramp-seconds", type=float, default=0.4,
                    help="untimed replays of the K steps before the timed region run for at "
                         "least this long (and >= 300 steps): HBM-bound steps speed up over "
                         "the first ~0.1-0.3 s of sustained work (profiles/r05/clock_replay.txt)")
    ap.add_argument("--workload", default="C", choices=sorted(WORKLOADS))
    ap.add_argument("--integrator", default=None,
                    choices=["rect+cum", "rect+rot", "rect", "qk21+rot", "qk21"],
                    help="kernel arithmetic (DESIGN.md 'Integrators'): qk21 = the reference's "
                         "quad() bit for bit, rect = direct h*f; +rot = heading carried as "
                         "(sin, cos) and rotated per step; +cum = rotated from the identity, "
                         "start pose applied last (enables chained steps, one launch per "
                         "step). Default: rect+cum for the episode workloads B/C/D, rect+rot "
                         "for E/F/G")
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="per-core time budget of the cpu_baseline sample (0 = skip)")
    ap.add_argument("--host-loop", action="store_true",
                    help="drive the episode from the host (one 808-B read + host update per "
                         "step) instead of the device-resident episode")
    ap.add_argument("--inputs", default="resident", choices=["resident", "sampled", "generated"],
                    help="resident: each step's candidates already in HBM (the contract's "
                         "input); sampled: the device sampler regenerates them per step")
    ap.add_argument("--no-second-pass", action="store_true",
                    help="skip the comparison run with the other --inputs mode")
    ap.add_argument("--layout", default="tiled", choices=["tiled", "soa"],
                    help="resident batches of the chained steps (one GPU, P2P): tiled = "
                         "MPC_LAYOUT_TILED (each 512-candidate tile's horizon contiguous in HBM, "
                         "include/mpc_rollout.h), soa = the step-major SoA every entry accepts")
    ap.add_argument("--no-config-d", action="store_true",
                    help="workload C: skip the config-D sub-results measured in the same run "
                         "(N=12; config_d: 1.25e6 candidates per GPU, weak; config_d_total: "
                         "1e7 in total over the N GPUs, strong — BASELINE's multi-GPU config)")
    ap.add_argument("--parity-steps", type=int, default=116,
                    help="chained episode workloads: after the timed regions, the checker "
                         "legs of parity_pass (oracle/parity.py) against the CPU oracle in "
                         "the reference's arithmetic (qk21): the line's `parity`.  One GPU: "
                         "this many steps of the episode leg (default 116: the reference's "
                         "events at p = 60 / 90 / 110 and a restart); 0 = skip every leg")
    ap.add_argument("--fused", action="store_true",
                    help="one launch per step: the rollout's last block runs the selection "
                         "(mpc_episode_rollout) instead of a separate selection launch")
    ap.add_argument("--no-chain", action="store_true",
                    help="separate selection launch per step instead of chained steps "
                         "(mpc_episode_chain_step: the step's launch completes the previous step)")
    ap.add_argument("--step-form", default="chain", choices=["run", "chain"],
                    help="one-GPU chained episode (rect+cum, resident batches): run = the K "
                         "steps as ONE persistent launch per 64 steps (mpc_episode_run: step "
                         "k+1 streams while step k is selected, no per-step kernel boundary, "
                         "no closing flush); chain = one chained launch per step + the flush")
    ap.add_argument("--no-graph", action="store_true",
                    help="time eagerly launched steps instead of a HIP graph replay")
    ap.add_argument("--exchange", action="store_true",
                    help="use the multi-GPU step structure (finalize -> RCCL all_gather -> "
                         "advance) even on one rank: rehearses the exchange and its graph "
                         "capture on a single GPU (1-rank process group)")
    ap.add_argument("--overlap-exchange", action="store_true",
                    help="exchange steps: run the all_gather of step k on a side stream beside "
                         "launch k+1, whose block 0 waits for the collective's device-side mark "
                         "(mpc_episode_exchange_step2) instead of the launch waiting for it")
    ap.add_argument("--exchange-mode", default="p2p", choices=["rccl", "p2p"],
                    help="chained exchange steps: rccl = one RCCL all_gather of the 536-B "
                         "candidates per step between the launches; p2p = no collective, each "
                         "launch's block 0 stores its candidate into every rank's mailbox over "
                         "xGMI (mpc_episode_p2p_step)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: rehearse N ranks on fewer GPUs (exchange staged via host)")
    ap.add_argument("--candidates-per-gpu", type=int, default=None,
                    help="override the workload's per-GPU candidate count")
    ap.add_argument("--dump-log", default=None,
                    help="write the device episode's per-step log (rank 0) to this JSON file")
    ap.add_argument("--traffic-json", default=None,
                    help="PMC-derived HBM bytes per launch for the roofline 'traffic' field "
                         "(tools/pmc.sh + tools/pmc_summary.py on the same kernel and config; "
                         "default: the committed round-2 summary of the roofline's kernel)")
    args = ap.parse_args()
    if args.integrator is None and args.workload in ("A", "R"):
        args.integrator = "qk21"          # the drop-in's default: the reference's arithmetic
    if args.integrator is None:
        args.integrator = "rect+cum" if args.workload in ("B", "C", "D") else "rect+rot"
    if args.warmup is None:
        args.warmup = 1 if args.workload == "A" else 5 if args.workload == "R" else 20
    if args.steps is None:
        args.steps = (50 if args.workload in ("F", "G") else 3 if args.workload == "A"
                      else 1000 if args.workload == "R" else 500)
    return args


def cpu_baseline_fulltree(seconds):
    """Config F: the C oracle of the full tree (oracle/mpc_oracle.c, qk21 and
    glibc trig as the reference) on one host core, S1 = 6 x 11 trees."""
    import math as _m
    import numpy as np
    from oracle import oracle as O
    V = np.round(np.arange(0, 1 + 0.2, 0.2), 3)
    B = np.round(np.linspace(-1.047, 1.047, 11), 3)
    n, leaves, t0 = 0, 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        O.fulltree_argmin(V, B, (0.1 * n, 0.0, 0.3), (4.0, 5.0), (0.0, 0.0),
                          float(np.arctan(4.0 / 5.0)), 0.5, 0.05, 0.1, 1e18)
        n += 1
        leaves += (len(V) * len(B)) ** 3
    dt = time.perf_counter() - t0
    return {"value": leaves / dt, "unit": "leaves/s", "cores": 1, "kind": "port",
            "sample": f"{n} full trees of S1 = {len(V) * len(B)} ({leaves} leaves), C oracle "
                      f"(qk21, glibc trig), {dt:.1f} s"}


def cpu_baseline(wl, seconds):
    """Reference-structured Python port on host cores (before GPU init)."""
    import numpy as np
    from diplomjourney_amd import math_model_tree as mmt
    from oracle import cpu_ref
    from oracle import oracle as O
    V = mmt.vector_of_velocities(0.0)
    B = mmt.vector_of_beta_angles(0.0)
    n_steps = wl["n_steps"]
    n = 400_000
    v, b = O.sample_controls(V, B, n, n_steps, seed=20261015 + 0x9E3779B9 * 1001)
    prob = (0.0, 0.0, 0.0, 2, 3, 0, 0, 0.5, 0.05, 0.1)
    r = cpu_ref.timed_rate(prob, v, b, budget_s=seconds)
    return {"value": r["rate"], "unit": "rollouts/s", "cores": r["cores"], "kind": "port",
            "affinity_cpus": r.get("affinity_cpus"), "cgroup_cpu_quota": r.get("cgroup_cpu_quota"),
            "sample": (f"{r['candidates']} sampled N={n_steps} candidates of the first MPC step "
                       f"(reference grid around v=0, beta=0), scipy.integrate.quad per "
                       f"integral as math_model_tree.py:91-115, {r['cores']} processes (every "
                       f"granted core: affinity {r.get('affinity_cpus')}, cgroup quota "
                       f"{r.get('cgroup_cpu_quota')}) x {seconds:.0f} s budget, busy "
                       f"{r['busy_s']:.1f} s")}


def _scenario_calls():
    """The reference's 349 recorded predictive_control calls (tests/golden,
    generated by running the reference; data only)."""
    with open(os.path.join(REPO, "tests", "golden", "reference_scenario.json")) as fh:
        return json.load(fh)["calls"]


def _call_controls(rec):
    """Candidate SoA [3, |V||B|] of one recorded call (slow-down :312-316)."""
    import numpy as np
    V, B = list(rec["V"]), list(rec["B"])
    if rec["pre"]["steps_for_slowing"] > 0:
        V = [min(V) if min(V) > 0.4 else 0.4] * len(V)
    vv = np.repeat(np.array(V, dtype=np.float64), len(B))
    bb = np.tile(np.array(B, dtype=np.float64), len(V))
    return np.tile(vv, (3, 1)), np.tile(bb, (3, 1))


def cpu_baseline_dropin(seconds):
    """Config A on one host core (the reference is single-threaded): the
    reference-structured port of predictive_control (oracle/cpu_ref.py,
    scipy.integrate.quad per integral, strict-< scan) on the recorded calls
    in order until the budget is spent — p50 of the expansion alone (the
    reference's own timer, :307 -> :362) and with the reference's
    CoordinateTree allocation of S1 + S1^2 + S1^3 object slots
    (CoordinateTree.py:5-9, freed after the call)."""
    import numpy as np
    from oracle import cpu_ref
    calls = _scenario_calls()
    exp_ms, e2e_ms, cands = [], [], 0
    t_start = time.perf_counter()
    for rec in calls:
        if time.perf_counter() - t_start > seconds:
            break
        v, b = _call_controls(rec)
        s1 = v.shape[1]
        pre, t = rec["pre"], rec["post"]["t"]
        prob = (rec["x"], rec["y"], rec["phi"], pre["x_t"], pre["y_t"], pre["x_0"], pre["y_0"],
                0.5, t, t + 0.05)
        t0 = time.perf_counter()
        tree = np.empty(s1 + s1 * s1 + s1 * s1 * s1, dtype=object)
        t1 = time.perf_counter()
        cpu_ref.expand(prob, v, b, 0, s1, incumbent=pre["optimal_criterion"])
        t2 = time.perf_counter()
        del tree
        t3 = time.perf_counter()
        exp_ms.append((t2 - t1) * 1e3)
        e2e_ms.append((t3 - t0) * 1e3)
        cands += s1
    from diplomjourney_amd.episode import percentile
    return {"value": percentile(e2e_ms, 50), "unit": "ms per MPC step (p50)", "cores": 1,
            "kind": "port", "p50_expansion_ms": percentile(exp_ms, 50),
            "rollouts_per_s_expansion": cands / (sum(exp_ms) * 1e-3),
            "sample": (f"the first {len(e2e_ms)} recorded reference calls ({cands} N=3 "
                       f"candidates), predictive_control's expansion as the reference runs it "
                       f"(scipy quad per integral) + its CoordinateTree allocation, one core")}


def bench_dropin(args, wl, eng, rank, world, cpu):
    """Config A: the reference scenario through the drop-in math_mpc /
    predictive_control (host episode loop, one C-ABI expansion + one 808-B
    read per call, as the reference calls it).  Parity against the recorded
    calls; p50 of predictive_control (host time, end to end) over --steps
    scenario runs after --warmup ones."""
    import torch
    from diplomjourney_amd import math_model_tree as mmt
    from diplomjourney_amd.episode import percentile
    mmt.INTEGRATOR = "qk21" if args.integrator is None else args.integrator
    calls = _scenario_calls()
    ms, rets = [], []
    orig = mmt.predictive_control

    def timed(*a):
        t0 = time.perf_counter()
        r = orig(*a)
        ms.append((time.perf_counter() - t0) * 1e3)
        rets.append(r)
        return r
    mmt.predictive_control = timed
    try:
        for _ in range(args.warmup):
            mmt.run_reference_scenario(seed=0)
        ms.clear()
        rets.clear()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            mmt.run_reference_scenario(seed=0)
        elapsed = time.perf_counter() - t0
    finally:
        mmt.predictive_control = orig
        mmt.reset_state()
    n_calls = len(rets)
    same = worst = 0
    for i, r in enumerate(rets):
        want = calls[i % len(calls)]["ret"]
        same += r[3:] == want[3:]
        worst = max(worst, max(abs(a - b) for a, b in zip(r[:3], want[:3])))
    cands = sum(len(c["V"]) * len(c["B"]) for c in calls) * args.steps
    out = {
        "metric": METRIC, "value": cands / elapsed, "unit": "rollouts/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / n_calls * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "the reference's own scenario (recorded inputs, tests/golden)",
        "config": {"workload": wl["desc"], "n_steps": 3, "calls_per_run": len(calls),
                   "integrator": mmt.INTEGRATOR if args.integrator is None else args.integrator,
                   "step": "drop-in predictive_control: host grid + candidate SoA upload, one "
                           "expansion launch pair (CoordinateTree states out), one 808-B read"},
        "p50_ms": percentile(ms, 50), "p90_ms": percentile(ms, 90),
        "p50_note": "host time per predictive_control call, end to end (the reference's "
                    "0.361 s p50 is the same call on one CPU core, SURVEY §6)",
        "parity": {"calls": n_calls, "chosen_control_identical": same,
                   "max_abs_pose_diff": worst},
        "roofline": None, "cpu_baseline": cpu,
    }
    if rank == 0:
        print(json.dumps(out), flush=True)


def visible_gpus():
    """GPUs this process could use, counted without touching the GPU or
    importing torch (the spawning parent stays GPU-free by construction):
    the KFD topology's GPU nodes (gpu_id != 0), narrowed by the visibility
    variables the HIP runtime honours.  0 when unknown (no check then)."""
    import glob
    n = 0
    for f in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/gpu_id"):
        try:
            with open(f) as fh:
                n += int(fh.read().strip() or 0) != 0
        except (OSError, ValueError):
            pass
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            ids = [x for x in v.split(",") if x.strip()]
            n = min(n, len(ids)) if n else len(ids)
    return n


def spawn_ranks(args):
    """`python bench.py --gpus N` (N > 1) without a launcher: this process
    stays GPU-free (it never initialises HIP: device counting does not) and
    starts N rank processes of this same script, one per GPU, with RANK /
    LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT in their
    environment — what `torch.distributed.run --nproc-per-node N` would do.
    Rank 0 prints the JSON line on the shared stdout.  If one rank fails the
    others are stopped; returns the worst exit status."""
    import signal
    import socket
    import subprocess
    n = args.gpus
    if args.dist_backend == "nccl":
        have = visible_gpus()
        if have and n > have:
            print(f"bench: --gpus {n} needs {n} GPUs for RCCL ranks ({have} visible); "
                  "--dist-backend gloo rehearses more ranks than GPUs", file=sys.stderr)
            return 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))

    def stop(*_):
        for p in procs:
            if p.poll() is None:
                p.terminate()
    signal.signal(signal.SIGTERM, lambda *a: (stop(), sys.exit(143)))
    worst = 0
    while any(p.poll() is None for p in procs):
        if any(p.returncode not in (None, 0) for p in procs):
            stop()
            t0 = time.time()
            while any(p.poll() is None for p in procs) and time.time() - t0 < 30:
                time.sleep(0.2)
            for p in procs:
                if p.poll() is None:
                    p.kill()
            break
        time.sleep(0.1)
    for p in procs:
        rc = p.wait()
        rc = 128 - rc if rc < 0 else rc     # killed by a signal: the shell's 128 + sig
        worst = max(worst, rc)
    return worst


def main():
    args = parse()
    wl = WORKLOADS[args.workload]
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus != world:
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU "
              f"(torch.distributed.run --nproc-per-node {args.gpus}) or run "
              f"`python bench.py --gpus {args.gpus}` without a launcher", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.print_ranks:     # launcher self-test (tests/test_host_logic.py): no GPU work
        print(json.dumps({"rank": rank, "local_rank": local_rank, "world": world,
                          "master": [os.environ.get("MASTER_ADDR"),
                                     os.environ.get("MASTER_PORT")]}), flush=True)
        return
    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        cpu = (cpu_baseline_fulltree(args.cpu_seconds) if args.workload in ("F", "G")
               else cpu_baseline_dropin(args.cpu_seconds) if args.workload in ("A", "R")
               else cpu_baseline(wl, args.cpu_seconds))

    import torch
    import torch.distributed as dist
    dev_index = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev_index)
    device = torch.device("cuda", dev_index)
    group = None
    if world > 1 or args.exchange:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=device)
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)
    n_dev = max(1, torch.cuda.device_count())
    if world > n_dev and args.workload in ("B", "C", "D"):
        # a rehearsal: several ranks share each GPU — each launches on its own
        # disjoint CU set, so that no rank's chained launch (tiles waiting for
        # block 0, which waits for the peers) takes the CUs a peer needs
        from diplomjourney_amd.episode import cu_share_stream
        torch.cuda.set_stream(cu_share_stream(device, local_rank // n_dev,
                                              -(-world // n_dev)))
    from diplomjourney_amd.expansion import Expansion
    eng = Expansion(device)

    if args.workload == "A":
        return bench_dropin(args, wl, eng, rank, world, cpu)
    if args.workload == "E":
        return bench_robots(args, wl, eng, rank, world, cpu)
    if args.workload == "R":
        return bench_tree_episodes(args, wl, eng, rank, world, cpu)
    if args.workload == "F":
        return bench_fulltree(args, wl, eng, rank, world, cpu)
    if args.workload == "G":
        return bench_episodes(args, wl, eng, rank, world, cpu)

    out, ep, pool = bench_episode(args, wl, eng, rank, world, device, cpu)
    chain = getattr(ep, "chain", False) and args.inputs == "resident" and not args.host_loop
    if chain and args.parity_steps > 0:
        # checker, after every timed region: logged steps re-scanned on the
        # host by the oracle in the reference's own arithmetic (qk21)
        out["parity"] = parity_pass(args, eng, ep, pool, rank, world, device)
    if args.workload == "C" and chain and not args.no_config_d:
        # BASELINE config D (N=12, 1.25e6 candidates per GPU = 1e7 at 8) in
        # the same run: at --gpus N the form the driver's scaling run measures
        ep_form = getattr(ep, "p2p", False)
        del pool
        finish_episode(ep)
        del ep
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        d_args = argparse.Namespace(**vars(args))
        d_args.candidates_per_gpu = None
        d_args.dump_log = None               # --dump-log is the main episode's
        d_out, ep, pool = bench_episode(d_args, WORKLOADS["D"], eng, rank, world, device, None,
                                        sub=True)
        out["config_d"] = {k: d_out[k] for k in (
            "value", "unit", "ms_per_step", "p50_ms", "chain_error", "exchange", "kernel_ms",
            "roofline", "roofline_valu")}
        out["config_d"]["config"] = {k: d_out["config"][k] for k in (
            "workload", "n_steps", "candidates_per_gpu", "candidates_total", "launch",
            "parallelism")}
        assert getattr(ep, "p2p", False) == ep_form or world == 1, "config D changed form"
        # BASELINE config D as written: 1e7 candidates IN TOTAL over the N
        # ranks (strong scaling: 1e7 on one GPU at N = 1, 1.25e6 per GPU at 8)
        del pool
        finish_episode(ep)
        del ep
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        t_args = argparse.Namespace(**vars(args))
        t_args.candidates_per_gpu = -(-D_TOTAL // world)
        t_args.dump_log = None
        t_out, ep, pool = bench_episode(t_args, WORKLOADS["D"], eng, rank, world, device, None,
                                        sub=True)
        out["config_d_total"] = {k: t_out[k] for k in (
            "value", "unit", "ms_per_step", "p50_ms", "p90_ms", "chain_error", "exchange",
            "kernel_ms", "roofline", "roofline_valu", "ramp")}
        out["config_d_total"]["scaling"] = "strong"
        out["config_d_total"]["config"] = {k: t_out["config"][k] for k in (
            "workload", "n_steps", "candidates_per_gpu", "candidates_total", "launch",
            "parallelism")}
        out["config_d_total"]["config"]["workload"] = (
            "config D as BASELINE.json states it: N=12, 1e7 candidates in total sharded over "
            "the N GPUs (contiguous index ranges; one exchange per step at N > 1)")
        out["config_d"]["scaling"] = "weak"
    if rank == 0:
        print(json.dumps(out, default=_plain), flush=True)
    finish(ep, world > 1 or args.exchange)


def _plain(o):
    """json default: numpy scalars (the checker's comparisons) as Python ones."""
    import numpy as np
    if isinstance(o, np.generic):
        return o.item()
    raise TypeError(f"not JSON serializable: {type(o).__name__}")


def bench_episode(args, wl, eng, rank, world, device, cpu, sub=False):
    """The episode workloads (B, C, D): returns (the JSON line's dict, the
    DeviceEpisode, its resident pool).  sub: a secondary workload of the same
    run (config D beside C) — no second input pass, no host latency pass."""
    import torch
    import torch.distributed as dist
    from diplomjourney_amd.episode import DeviceEpisode, Episode, cu_reserved_stream, percentile
    group = None
    n_total = (args.candidates_per_gpu or wl["per_gpu"]) * world
    n_steps = wl["n_steps"]
    exchange = world > 1 or args.exchange
    overlap = args.overlap_exchange and exchange and not args.host_loop
    p2p = (args.exchange_mode == "p2p" and exchange and not args.host_loop and not overlap
           and not args.no_chain and args.integrator == "rect+cum" and args.inputs == "resident")
    if overlap:
        # the steps' launch stream leaves one CU per XCD to the collective that
        # runs beside each launch (RCCL's kernel never fits beside a full CU)
        torch.cuda.set_stream(cu_reserved_stream(device, 1))
    # one GPU: the K steps are one HIP graph; with the exchange the RCCL
    # all_gather is captured into the same graph (gloo stages through the
    # host and cannot be captured)
    # (the overlapped exchange launches eagerly: a replayed graph's parallel
    # branches lose the launch stream's CU mask)
    use_graph = (not args.host_loop and not args.no_graph and not overlap
                 and (not exchange or p2p or args.dist_backend == "nccl"))
    inputs = "sampled" if args.host_loop else args.inputs
    if args.host_loop:
        ep = Episode(eng, n_total, n_steps, rank=rank, world=world,
                     integrator=args.integrator, group=group)
    else:
        ep = DeviceEpisode(eng, n_total, n_steps, rank=rank, world=world,
                           integrator=args.integrator, group=group, log_capacity=8192,
                           exchange=exchange, split=not args.fused,
                           chain=not args.no_chain and args.integrator == "rect+cum",
                           generate=inputs == "generated",
                           overlap=overlap, p2p=p2p)
        p2p = bool(getattr(ep, "p2p", False))    # (False if its self-test failed)
    # the chained steps stream tiled batches (one GPU and P2P forms)
    tiled = (args.layout == "tiled" and inputs == "resident" and not args.host_loop
             and getattr(ep, "chain", False) and (not exchange or p2p))
    pool = make_pool(eng, ep, n_steps, args.steps, tiled) if inputs == "resident" else None
    rollout_ms = None
    # the launch that carries the step: the chained kernel (rollout of step k +
    # completion of step k-1; on G > 1 its exchange form, which also selects
    # over the gathered candidates and collects this rank's) or the rollout kernel
    chained = not exchange and getattr(ep, "chain", False) and inputs == "resident"
    xchg_chain = exchange and getattr(ep, "chain", False) and inputs == "resident"
    # one GPU: the K steps as one persistent run (mpc_episode_run) by default
    run_form = chained and args.step_form == "run" and hasattr(ep, "run")
    kernel = ("k_episode_run" if run_form else "k_episode_chain" if chained
              else (P2P_KERNEL if p2p else XCHG_KERNEL) if xchg_chain
              else "k_rollout_argmin_stream")
    main_run = run_steps(args, ep, pool, use_graph, world, device, run_form=run_form)
    use_graph = main_run["graph"]
    kern_ms = main_run["kernel_in_step_ms"]
    sustained_ms = None
    if run_form and use_graph:
        # the run's device time per step inside the timed replay; sustained:
        # a 200-step run replayed (reported beside it)
        kern_ms = main_run["kernel_timed_ms"]
        sustained_ms = None if sub else run_pass(ep, pool)
    elif run_form:
        kern_ms = run_pass(ep, pool)
    elif (chained or (xchg_chain and p2p)) and use_graph:
        # one launch per step, the K of the timed region back to back: HIP
        # events around them inside the timed replay
        kern_ms = main_run["kernel_timed_ms"]
        # the same launches sustained over a longer run (200 eager + 2 x 200
        # replayed; reported beside the timed region's value)
        sustained_ms = None if sub else chain_pass(ep, pool)
    elif chained or (xchg_chain and p2p):
        kern_ms = chain_pass(ep, pool)
    elif xchg_chain:
        # the all_gather form has its collective between two launches: a pair
        # of events per launch
        kern_ms = exchange_chain_pass(ep, pool)
    elif inputs == "generated":
        pass   # events around the generated rollout + selection (no HBM roofline)
    elif hasattr(ep, "partials"):
        kern_ms = kernel_pass(ep, pool if pool is not None else
                              make_pool(eng, ep, n_steps, 4))
    if chained and not sub:
        # for comparison: the same controls through the rollout kernel alone
        # (the chained launch adds block 0's completion of the previous step)
        rollout_ms = kernel_pass(ep, soa_pool(ep, pool))
    other = generated = None
    if not args.host_loop and not args.no_second_pass and not sub:
        # the other input mode, same episode machinery, for comparison
        other_pool = None if inputs == "resident" else make_pool(eng, ep, n_steps, args.steps)
        # (gloo collectives stage through the host: not capturable)
        r = run_steps(args, ep, other_pool,
                      use_graph and not (exchange and args.dist_backend == "gloo"), world, device)
        other = {"inputs": "sampled" if inputs == "resident" else "resident",
                 "value": n_total * args.steps / r["elapsed"],
                 "ms_per_step": r["elapsed"] / args.steps * 1e3, "p50_ms": r["p50_ms"]}
        del other_pool
        if inputs == "resident" and not exchange:
            # the sampled candidates drawn inside the rollout instead (one GPU)
            ep.generate = True
            r = run_steps(args, ep, None, use_graph, world, device)
            ep.generate = False
            generated = {"inputs": "generated", "value": n_total * args.steps / r["elapsed"],
                         "ms_per_step": r["elapsed"] / args.steps * 1e3,
                         "p50_ms": r["p50_ms"],
                         "roofline_valu": valu_roofline(
                             "k_rollout_generated", args.integrator,
                             r["elapsed"] / args.steps * 1e3, n_total // world, n_steps,
                             note="over the whole step (generated rollout + selection): a "
                                  "lower bound of the rollout kernel's rate")}
    host_ms = None
    if not args.host_loop and not exchange and not sub:
        host_ms = host_latency_pass(ep, pool)
    elapsed = main_run["elapsed"]
    chain_step = getattr(ep, "chain", False) and inputs == "resident"
    bytes_launch = 16.0 * n_steps * ep.n_local
    achieved = bytes_launch / (kern_ms * 1e-3) / 1e9
    value = n_total * args.steps / elapsed
    # self-validation: a chained / exchange step whose bounded device wait
    # timed out ran on speculated constants or dropped a rank's candidate —
    # such a run reports no throughput (max over ranks; exit status 3)
    chain_err, log = 0, None
    if not args.host_loop:
        from diplomjourney_amd.episode import ChainError
        try:
            log = ep.read_log()
        except ChainError as e:
            chain_err = e.code
    chain_err = int(max_over_ranks(chain_err, device))
    if chain_err:
        from diplomjourney_amd.episode import CHAIN_ERRORS
        print(f"bench: chain_error {chain_err} on some rank: "
              f"{CHAIN_ERRORS.get(chain_err, 'unknown')}; no result", file=sys.stderr, flush=True)
        if dist.is_initialized():
            dist.destroy_process_group()
        sys.exit(3)
    if not args.host_loop:
        if args.dump_log and rank == 0:
            with open(args.dump_log, "w") as fh:
                json.dump([{f: getattr(r, f) for f, _ in r._fields_} for r in log], fh)
        assert len(log) == min(ep.steps_enqueued, ep.log_capacity), (len(log), ep.steps_enqueued)
        missing = [r.step for r in log if r.index < 0]
        assert not missing, f"steps without a winner: {missing[:20]}"
        episodes = log[-1].episode
    else:
        episodes = ep.episodes
    out = {
        "metric": METRIC, "value": value, "unit": "rollouts/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ramp": {"steps": main_run["ramp_steps"], "seconds": main_run["ramp_s"],
                 "note": "untimed replays of the K steps after the W warmup steps and before "
                         "the timed region (>= 300 steps and >= --ramp-seconds): the GPU's "
                         "clocks ramp over the first ~0.1-0.3 s of sustained work "
                         "(profiles/r05/clock_replay.txt); the timed region is sustained state"},
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": wl["desc"], "n_steps": n_steps,
                   "candidates_per_gpu": ep.n_local, "candidates_total": n_total,
                   "integrator": args.integrator, "inputs": INPUTS_DOC[inputs],
                   "layout": (LAYOUT_DOC["tiled"] if tiled else LAYOUT_DOC["soa"])
                   if inputs == "resident" else None,
                   "episodes_started": episodes,
                   "episode_loop": "host" if args.host_loop else "device-resident",
                   "launch": (("hipGraph of the K steps" + (" incl. the RCCL all_gather"
                                                            if exchange and not p2p else ""))
                              if use_graph else "eager"),
                   "step_launches": (
                       "persistent run: the K steps in ONE launch per 64 steps "
                       "(mpc_episode_run) — units (step, 512-candidate tile) claimed in order, "
                       "step k+1 streaming while block 0 selects and applies step k, the last "
                       "step completed inside the launch" if run_form else
                       ("chained: rollout of step k + completion of step k-1 in one launch"
                        + (" (selection over the gathered candidates of step k-1; the launch "
                           "also collects this rank's candidate of step k), "
                           + ("which block 0 stores into every rank's mailbox (peer stores; "
                              "no collective)" if p2p else "then the all_gather")
                           if exchange else "")
                        + (" on a side stream beside the next launch, whose block 0 waits for "
                           "its device-side mark; launches on a CU-masked stream (1 CU per XCD "
                           "left to the collective)" if overlap else ""))
                       if chain_step
                       else "rollout, then selection" + (
                           " + all_gather + advance" if exchange else "")),
                   "parallelism": f"candidate-sharded x{world}" + (
                       (", 536-B candidates by peer stores/step" if p2p
                        else ", all_gather(536 B candidates)/step" if chain_step
                        else ", all_gather(808 B)/step") if exchange else "")},
        "p50_ms": main_run["p50_ms"], "p90_ms": main_run["p90_ms"],
        "p50_note": "GPU time per MPC step (HIP events between step starts, eager launches)",
        "p50_host_ms": percentile(host_ms, 50) if host_ms else None,
        "p90_host_ms": percentile(host_ms, 90) if host_ms else None,
        "p50_host_note": ("host time per eager MPC step until its 808-B result record is in "
                          "pinned host memory (step launches + completion + D2H + sync), as a "
                          "controller receives the chosen control (math_model_tree.py:429); "
                          "reference: 0.361 s p50 per predictive_control at N=3, 451 "
                          "candidates (SURVEY §6)"),
        "exchange": (None if not exchange else getattr(ep, "p2p_status", None)
                     or ("all_gather (RCCL)" if args.dist_backend == "nccl"
                         else "all_gather (gloo)")),
        "chain_error": chain_err,
        "kernel_ms": kern_ms, "kernel_in_step_ms": main_run["kernel_in_step_ms"],
        "kernel_ms_note": ("device time per step inside the timed region (HIP events around "
                           "the timed graph replay of the K-step run, over K)" if run_form and
                           use_graph else
                           "device time per step launch inside the timed region (HIP events "
                           "around the timed graph replay, minus the closing flush's own "
                           "duration %.4f ms, over K)" % main_run["flush_ms"]
                           if (chained or (xchg_chain and p2p)) and use_graph
                           else "events around back-to-back launches (graph_timed / per launch)"),
        "kernel_ms_sustained": sustained_ms,
        "roofline": (None if inputs == "generated" else
                     roofline(achieved, bytes_launch, args.traffic_json, kernel=kernel,
                              layout="tiled" if tiled else "soa")),
        "roofline_rollout_only": (None if rollout_ms is None else
                                  roofline(bytes_launch / (rollout_ms * 1e-3) / 1e9, bytes_launch,
                                           None, kernel="k_rollout_argmin_stream")),
        "roofline_valu": valu_roofline(kernel, args.integrator, kern_ms, n_total // world,
                                       n_steps),
        "other_inputs": other,
        "generated_inputs": generated,
        "cpu_baseline": cpu,
    }
    if out["roofline"] is not None and pool is not None:
        # the same kernel against the measured read ceiling of
        # its own access pattern and its VALU issue share (PMC counters of the
        # committed traffic summary)
        ceil, ceil_ms = stream_ceiling(ep, pool)
        out["roofline"]["stream_ceiling_GBs"] = ceil
        out["roofline"]["stream_ceiling_ms"] = ceil_ms
        out["roofline"]["frac_of_stream_ceiling"] = achieved / ceil
        out["roofline"]["valu"] = valu_share(args.traffic_json, kernel, bytes_launch, kern_ms,
                                             out["roofline"].get("layout", "soa"))
    return out, ep, pool


def parity_pass(args, eng, ep, pool, rank, world, device):
    """CHECKER, run after every timed region and never timed: the hot path's
    forms of this run against the CPU oracle in the reference's arithmetic
    (qk21: scipy quad's 21-point Kronrod sums, glibc trig, the reference's
    operation order — oracle/mpc_oracle.c, pinned bitwise to the reference's
    own outputs).  Legs (oracle/parity.py):
      episode      a fresh device episode of the bench's own step form (same
                   shard, chained launch, layout and exchange) over the first
                   resident batches, through the operator events and a
                   restart (one GPU: the reference schedule p = 60 / 90 / 110
                   with a step limit of 112, 116 steps; N > 1: p = 6 / 12 / 16,
                   limit 20, 24 steps), against an INDEPENDENT oracle episode
                   that scans each batch itself from ITS OWN previous winner:
                   index, (v, beta), returned pose, status bits per step
                   (math_model_tree.py:351-359,392-414,542-569);
      sampler      the first resident batch (tiled sampler) and 3 steps of a
                   sampled-mode episode (the device sampler on the grid around
                   the chosen control), bitwise against the oracle sampler,
                   and those steps' winners (:239-256,312-316);
      fulltree     one S1 = 451 full-tree step (run_math_model.py:156-197),
                   device qk21 and rect+rot vs the oracle's scan;
      ft_episodes  8 of run_math_model.py's episodes (:231-280), device
                   resident (mpc_fulltree_episodes_run) vs the oracle;
      tree_episodes the named entry over the tree expansion (mpc_episodes_run)
                   vs the oracle.
    Every rank checks its own shard; the ranks' lexicographic (cost, index)
    minima give the oracle's global winner."""
    import math as _m
    import numpy as np
    import torch
    import torch.distributed as dist
    from oracle import parity as P
    from diplomjourney_amd import math_model_tree as mmt
    from diplomjourney_amd.episode import DeviceEpisode
    t_start = time.perf_counter()
    try:
        threads = max(1, min(16, len(os.sched_getaffinity(0)) // max(1, world)))
    except AttributeError:
        threads = 4
    on_dev = dist.is_initialized() and dist.get_backend() == "nccl"

    def allgather(a):
        a = np.ascontiguousarray(a, dtype=np.float64)
        if world == 1:
            return a[None]
        t = torch.from_numpy(a).to(device if on_dev else "cpu")
        outs = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(outs, t)
        return np.stack([o.cpu().numpy() for o in outs])

    # -- episode: the bench's own chained form through events and a restart --
    if world == 1:
        sched = dict(p_turn_right=60, p_turn_left=90, p_new_target=110, max_steps=112)
        K = args.parity_steps if args.parity_steps > 0 else 116
    else:
        sched = dict(p_turn_right=6, p_turn_left=12, p_new_target=16, max_steps=20)
        K = 24
    nb = min(8, len(pool))
    fresh = DeviceEpisode(eng, ep.n_total, ep.n_steps, rank=rank, world=world,
                          integrator=ep.integrator, group=ep.group, log_capacity=max(64, K),
                          exchange=ep.exchange, chain=True, p2p=getattr(ep, "p2p", False),
                          max_steps=sched["max_steps"])
    for k, v in sched.items():
        setattr(fresh.cfg, k, v)
    fresh.reset()                        # the state takes the schedule
    if world == 1 and not ep.exchange and args.step_form == "run":
        fresh.run([pool[i % nb] for i in range(K)])    # the bench's persistent run
    else:
        for i in range(K):
            fresh.step(controls=pool[i % nb])
        fresh.flush()
    log = fresh.read_log()
    cfg = fresh.cfg
    finish_episode(fresh)
    del fresh
    host = [(v.cpu().numpy(), b.cpu().numpy()) for v, b in soa_pool(ep, pool, nb)]
    scanners = [P.ShardScanner(v, b, ep.lo, threads) for v, b in host]
    out = {"episode": P.episode_leg((cfg, log), None, scanners, allgather, threads)}
    out["episode"]["schedule"] = sched
    del scanners

    # -- sampler: the resident batch, then sampled-mode steps -----------------
    V0 = mmt.vector_of_velocities(0.5)
    B0 = mmt.vector_of_beta_angles(0.0)
    ov, ob = O_sample(V0, B0, ep.n_local, ep.n_steps, 0x5EED0000, ep.lo)
    pool_bitwise = bool(np.array_equal(ov, host[0][0]) and np.array_equal(ob, host[0][1]))
    del host, ov, ob
    samp = DeviceEpisode(eng, ep.n_total, ep.n_steps, rank=rank, world=world,
                         integrator=ep.integrator, group=ep.group, log_capacity=64,
                         exchange=ep.exchange, chain=False)
    drawn = []
    for _ in range(3):
        samp.step()
        drawn.append((samp.v_sc.cpu().numpy(), samp.b_sc.cpu().numpy()))
    slog = samp.read_log()
    s = P.sampled_leg(samp.cfg, drawn, slog, ep.n_local, ep.n_steps, ep.lo, allgather, threads)
    finish_episode(samp)
    del samp, drawn
    s["resident_batch_bitwise"] = bool(np.all(allgather(np.array([float(pool_bitwise)])) == 1.0))
    out["sampler"] = s

    # -- full tree: one S1 = 451 step (workload F's grid and first call) ------
    from diplomjourney_amd import run_math_model as rmm
    from diplomjourney_amd.abi import MpcFulltreeProblem
    from diplomjourney_amd.expansion import fulltree_argmin, fulltree_result
    rmm.configure(0.1, _m.radians(3))
    try:
        Vf, Bf = np.asarray(rmm.vector_v, dtype=np.float64), np.asarray(rmm.vector_beta,
                                                                        dtype=np.float64)
        st, tg = (-3.0, -2.0, 0.3), (4.0, 5.0)
        atan_t = float(np.arctan(tg[0] / tg[1]))
        inc = P._ft_criterion0(*st, *tg)
        vg = torch.tensor(Vf, device=eng.device)
        bg = torch.tensor(Bf, device=eng.device)
        fp = MpcFulltreeProblem(*st, *tg, st[0], st[1], atan_t, float(rmm.L), 0.05, 0.1)
        dev = {}
        for integ in ("qk21", "rect+rot"):
            r = fulltree_result(fulltree_argmin(eng, fp, vg, bg, inc, integ))
            dev[integ] = (r.leaf, r.cost, r.found, r.trajectory())
        out["fulltree"] = P.fulltree_leg(dev, Vf, Bf, (st, tg, st[:2], atan_t, float(rmm.L),
                                                       0.05, 0.1), inc, rank, world, allgather,
                                         threads)
        # -- the script's episodes, device resident (workload G's grid) -------
        rmm.configure(0.25, _m.radians(10))
        starts = rmm.draw_starts(8, seed=20261015)
        t0 = time.perf_counter()
        ref = P.ft_episodes_oracle(starts, np.asarray(rmm.vector_v, dtype=np.float64),
                                   np.asarray(rmm.vector_beta, dtype=np.float64), float(rmm.L),
                                   float(rmm.delta_t), float(rmm.eps), 4, threads)
        fe = {}
        for integ in ("qk21", "rect+rot"):
            d = rmm.run_batched(starts, max_calls=4, integrator=integ)
            fe[integ] = P.compare_episodes(
                [([r["ret"] + [r["optimal_criterion"]] for r in recs], stop) for recs, stop in d],
                ref)
        fe["s1"] = int(rmm.size_max_1)
        fe["check_s"] = time.perf_counter() - t0
        out["ft_episodes"] = fe
    finally:
        rmm.configure()
    # -- the named entry over the tree expansion (workload R's engine) -------
    starts = rmm.draw_starts(8, seed=20261016)
    t0 = time.perf_counter()
    d = rmm.run_tree_batched(starts, max_calls=12, integrator="qk21", engine=eng)
    te = P.compare_episodes(d, P.tree_episodes_oracle(starts, 12, threads))
    te["check_s"] = time.perf_counter() - t0
    out["tree_episodes"] = te

    e, sm, ft = out["episode"], out["sampler"], out["fulltree"]
    fq = out["ft_episodes"]["qk21"]
    checks = {
        "episode_identity": e["identity_rate"] == 1.0,
        "episode_v_beta": e["v_beta_identical_rate"] == 1.0,
        "episode_pose_le_1e-6": e["max_abs_pose_diff"] <= 1e-6,
        "episode_status": e["status_identical_rate"] == 1.0 and e["p_episode_identical_rate"] == 1.0,
        "episode_events_and_restart": e["event_steps"] >= 1 and e["restarts"] >= 1,
        "sampler_bitwise": sm["batches_bitwise"] and sm["resident_batch_bitwise"],
        "sampled_identity": sm["identity_rate"] == 1.0 and sm["max_abs_pose_diff"] <= 1e-6,
        "fulltree_qk21": ft["qk21"]["leaf_identical"] and ft["qk21"]["max_abs_state_diff"] <= 1e-9,
        "ft_episodes_qk21": (fq["stops_identical"] and fq["calls_identical"]
                             and fq["v_beta_identical_rate"] == 1.0
                             and fq["max_abs_pose_diff"] <= 1e-9),
        "tree_episodes_qk21": (te["stops_identical"] and te["calls_identical"]
                               and te["v_beta_identical_rate"] == 1.0
                               and te["max_abs_pose_diff"] <= 1e-9),
    }
    out.update({
        "steps": e["steps"], "identity_rate": e["identity_rate"],
        "max_abs_pose_diff": e["max_abs_pose_diff"], "checks": checks,
        "pass": all(checks.values()),
        "oracle": "qk21 (the reference's scipy quad arithmetic), oracle/mpc_oracle.c; episode "
                  "bookkeeping restated in oracle/parity.py",
        "threads_per_rank": threads, "check_s": time.perf_counter() - t_start,
        "note": "checker after the timed regions, not part of any timed value; rect+rot rows "
                "are the kernels' other arithmetic against the same qk21 oracle (reported, "
                "not gated)"})
    return out


def O_sample(V, B, n, n_steps, seed, lo):
    """The oracle sampler (checker only)."""
    from oracle import oracle as O
    return O.sample_controls(V, B, n, n_steps, seed, index_base=lo)


def finish_episode(ep):
    """An episode done with: drain it and release its mailbox (every rank)."""
    import torch
    import torch.distributed as dist
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.barrier()       # no peer still stores into this rank's mailbox
    close = getattr(ep, "close", None)
    if close:
        close()
    torch.cuda.synchronize()


def finish(ep, have_group):
    """Drain everything this run enqueued (peer stores, a side stream's last
    collective), release the episode's mailbox, then the process group — so
    nothing is in flight when the runtime tears down at exit."""
    import torch.distributed as dist
    finish_episode(ep)
    if have_group and dist.is_initialized():
        dist.destroy_process_group()


def stream_ceiling(ep, pool, reps=200, warm=100):
    """Measured read ceiling of the rollout's own access pattern on this GPU:
    mpc_stream_probe (the streaming kernel's grid, tiles and LDS-DMA control
    ring, no arithmetic; mpc_stream_probe_tiled for tiled batches) over the
    same resident batches, REPS back-to-back launches replayed from a HIP
    graph (graph_timed), rotating over the pool as kernel_pass does.  Returns (GB/s of the 16 B per candidate-step
    read, ms per launch)."""
    import ctypes
    import torch
    lib = ep.lib
    n, ns = ep.n_local, ep.n_steps
    sink = torch.empty(2048 * 256, dtype=torch.int64, device=pool[0][0].device)

    def one(i):
        # (the current stream at each launch: graph_timed captures on its own)
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        p = pool[i % len(pool)]
        if isinstance(p, torch.Tensor):      # tiled: the chained kernel's tiled pattern
            rc = lib.mpc_stream_probe_tiled(p.data_ptr(), n, ns, sink.data_ptr(),
                                            sink.numel() * 8, st)
        else:
            v, b = p
            rc = lib.mpc_stream_probe(v.data_ptr(), b.data_ptr(), n, ns, sink.data_ptr(),
                                      sink.numel() * 8, st)
        if rc != 0:
            raise RuntimeError(f"mpc_stream_probe: status {rc}")
    ms, _ = graph_timed(one, reps, warm)
    return 16.0 * ns * n / (ms * 1e-3) / 1e9, ms


def host_latency_pass(ep, pool, n=200):
    """The latency a controller sees (the reference returns the chosen
    control to its caller every step, math_model_tree.py:429): per eager MPC
    step, host time from enqueueing the step until its 808-B result record is
    in pinned host memory — the step's launches (a chained step is completed
    by its flush launch), the D2H copy and the stream sync.  Episode state
    stays on the device; returns the per-step host times in ms."""
    import torch
    host = torch.empty(ep.local.numel(), dtype=torch.uint8).pin_memory()
    stream = torch.cuda.current_stream()
    out = []
    for i in range(n + 20):
        t0 = time.perf_counter()
        if pool is None:
            ep.step()
        else:
            ep.step(controls=pool[i % len(pool)])
        ep.flush()
        host.copy_(ep.local, non_blocking=True)
        stream.synchronize()
        if i >= 20:
            out.append((time.perf_counter() - t0) * 1e3)
    return out


def valu_share(traffic_json, kernel, bytes_launch, kern_ms, layout="soa"):
    """VALU wave-instructions per launch (SQ_INSTS_VALU, PMC) and the share of
    the fp64 issue rate they take: 4 cycles per wave-instruction on each of the
    1024 SIMDs at 2.4 GHz (78.6 TFLOP/s of fp64 FMA); integer and fp32 VALU
    instructions are counted as fp64 ones, so the share is an upper bound."""
    t, path = traffic_summary(traffic_json, kernel, bytes_launch, layout)
    insts = t.get("counters_median_per_launch", {}).get("SQ_INSTS_VALU") if t else None
    if insts is None:
        return None
    return {"wave_insts_per_launch": insts, "source": os.path.relpath(path, REPO),
            "fp64_issue_share": insts * 4.0 / (1024 * 2.4e9 * kern_ms * 1e-3)}


INPUTS_DOC = {
    "resident": "per step a distinct synthetic candidate batch already in HBM (generated "
                "before the timed region by the device sampler: reference grid around "
                "v=0.5, beta=0, const-control prefix); the step = rollout/arg-min + "
                "finalize/episode update.  It does NOT regenerate the grid around the "
                "step's chosen control as the reference does (math_model_tree.py:543-545): "
                "that is the sampled / generated modes (other_inputs / generated_inputs)",
    "sampled": "per step the device sampler regenerates the candidates on the grid around "
               "the episode's current control (the reference's per-step grid); the step = "
               "sampler + rollout/arg-min + finalize/episode update",
    "generated": "the sampled mode's candidates drawn inside the rollout kernel (grid in LDS, "
                 "the sampler's hash per candidate-step; never written to HBM); the step = "
                 "generated rollout/arg-min + finalize/episode update",
}


def make_pool(eng, ep, n_steps, k, tiled=False):
    """Distinct resident candidate batches for the timed steps (cycled when
    K batches would exceed ~16 GB; at least 4, so a batch is never
    cache-resident when it comes round again).  tiled: MPC_LAYOUT_TILED
    tensors (the same candidates as the SoA batches of the same seeds)."""
    import torch
    from diplomjourney_amd import math_model_tree as mmt
    batch = 16 * n_steps * ep.n_local
    n = max(1, min(k, max(4, int(16e9 // batch))))
    V = torch.tensor(mmt.vector_of_velocities(0.5), dtype=torch.float64, device=eng.device)
    B = torch.tensor(mmt.vector_of_beta_angles(0.0), dtype=torch.float64, device=eng.device)
    if tiled:
        pool = [eng.sample_controls_tiled(V, B, ep.n_local, n_steps, 0x5EED0000 + i,
                                          index_base=ep.lo) for i in range(n)]
    else:
        pool = [eng.sample_controls(V, B, ep.n_local, n_steps, 0x5EED0000 + i, index_base=ep.lo)
                for i in range(n)]
    torch.cuda.synchronize()
    return pool


def soa_pool(ep, pool, k=4):
    """The first k batches as SoA (v, beta) pairs (tiled batches converted):
    for the passes that read the ABI's step-major layout (the streaming kernel
    alone, the host checker)."""
    import torch
    from diplomjourney_amd.expansion import tiled_to_soa
    out = [tiled_to_soa(p, ep.n_local) if isinstance(p, torch.Tensor) else p for p in pool[:k]]
    return out


LAYOUT_DOC = {
    "tiled": "MPC_LAYOUT_TILED: each 512-candidate tile's v and beta of every step in one "
             "contiguous run (include/mpc_rollout.h); 16 B per candidate-step as in SoA",
    "soa": "step-major SoA v_sc[s * C + c], beta_sc[s * C + c]",
}


def run_steps(args, ep, pool, use_graph, world, device, run_form=False):
    """Warmup, the timed K steps, then the eager latency passes.

    With a graph (the default): the K steps — and a chained episode's closing
    flush — are captured once into ONE graph (one replay call: the least host
    launch overhead in a short timed region), replayed untimed until ~300
    steps have run (the GPU's clocks ramp over the first few hundred
    launches), then replayed ONCE between barrier + sync on both sides (host
    clock: `elapsed`, the value's denominator) with HIP events around the
    replay on the launch stream.  `kernel_timed_ms` = (that event time - the
    closing flush's own duration, measured eagerly afterwards) / K: the device
    time per step launch inside the timed region (for chained steps the
    chained kernel back to back — the roofline's denominator).  Then, eagerly:
    K steps with one event per step start (p50 / p90 of the GPU time per step)
    and up to 20 steps with events around the step's launch
    (`kernel_in_step_ms`)."""
    import torch
    import torch.distributed as dist
    from diplomjourney_amd.episode import percentile

    def step(i, events=None):
        if run_form:                       # one complete step: a run of one
            if events:
                events[0].record()
            ep.run([pool[i % len(pool)]])
            if events:
                events[1].record()
        elif pool is None:
            ep.step(events=events)
        else:
            ep.step(events=events, controls=pool[i % len(pool)])

    def steps_k():
        if run_form:                       # the K steps: ONE persistent run
            ep.run([pool[i % len(pool)] for i in range(args.steps)])
        else:
            for i in range(args.steps):
                step(i)

    flush = getattr(ep, "flush", lambda: None)   # completes a chained step left pending
    Ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    for i in range(args.warmup):
        step(i)
    flush()
    torch.cuda.synchronize()
    graph = None
    if use_graph:
        n0 = ep.steps_enqueued
        try:
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                steps_k()
                flush()                      # the K-th step completes inside the graph
        except Exception as e:   # capture refused (e.g. by the collective): launch eagerly
            print(f"bench: graph capture failed ({type(e).__name__}: {e}); eager launches",
                  file=sys.stderr, flush=True)
            graph = None
            if hasattr(ep, "_pending"):
                ep._pending = None           # the captured launches never ran
            torch.cuda.synchronize()
        ep.steps_enqueued = n0               # captured, not run

    def run_k():
        if graph is not None:
            graph.replay()
            ep.steps_enqueued += args.steps
        else:
            steps_k()
            flush()

    # untimed: the clock ramp. At least 300 steps and ramp_seconds of wall
    # time; the host waits every ~2 ms of queued work so that it never runs
    # far ahead of the GPU. Repeated K=20 replays, each after a sync, take
    # 33-34 us per step for the first ~0.1-0.3 s of a process's work and
    # 28.5-29 after it (profiles/r05/clock_replay.txt).
    # Every rank runs the same number of replays (the exchange steps are
    # collective): the ranks agree on going on (MAX of their flags).
    ran, t_ramp = 0, time.perf_counter()
    while True:
        for _ in range(max(1, 64 // args.steps)):
            run_k()
            ran += args.steps
        torch.cuda.synchronize()
        more = ran < 300 or time.perf_counter() - t_ramp < getattr(args, "ramp_seconds", 0.0)
        if world > 1:
            f = torch.tensor([1.0 if more else 0.0], dtype=torch.float64, device=device)
            dist.all_reduce(f, op=dist.ReduceOp.MAX)
            more = float(f.item()) > 0
        if not more:
            break
    # one more untimed replay, waited for at once: the host's last wait before
    # the timed region is then one replay long, not the ~10 ms of the warm
    # replays — after a long blocking wait the timed replay's launches reach
    # the GPU late (kernel trace: 28-31.5 us kernels starting 34-38 us apart).
    # Same box, 4 interleaved pairs at K = 20: 33.0-33.6 vs 33.5-34.3 us per
    # step (profiles/r05/driver_ab.txt)
    run_k()
    ran += args.steps
    torch.cuda.synchronize()
    ramp_s = time.perf_counter() - t_ramp
    # no collector pass inside the timed region: after the checker legs the
    # heap holds many objects, and one full collection took ~6 ms of a 12-ms
    # timed region (config_d_total at K = 20: 0.59 ms/step host time against
    # 0.29 ms of kernel time by events; 0.296 standalone)
    gc.collect()
    gc.disable()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    e0, e1 = Ev(), Ev()
    t0 = time.perf_counter()
    e0.record()
    run_k()
    e1.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    gc.enable()
    timed_ms = e0.elapsed_time(e1)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # latency pass: one event per step start (more events per step would add
    # their own host cost to an eagerly launched step)
    marks = [Ev() for _ in range(args.steps + 1)]
    torch.cuda.synchronize()
    for i in range(args.steps):
        marks[i].record()
        step(i)
    marks[-1].record()
    flush()
    torch.cuda.synchronize()
    step_gpu_ms = [marks[i].elapsed_time(marks[i + 1]) for i in range(args.steps)]
    # the step's launch inside eager steps, events around it; and the closing
    # flush's own duration (a pending chained step completed alone)
    n_kern = min(args.steps, 20)
    kern = [(Ev(), Ev()) for _ in range(n_kern)]
    fl = [(Ev(), Ev()) for _ in range(n_kern)]
    has_flush = False
    for i in range(n_kern):
        step(i, kern[i])
        has_flush = has_flush or getattr(ep, "_pending", None) is not None
        fl[i][0].record()
        flush()
        fl[i][1].record()
    torch.cuda.synchronize()
    flush_ms = (sum(a.elapsed_time(b) for a, b in fl) / n_kern) if has_flush else 0.0
    return {"elapsed": elapsed, "graph": graph is not None, "ramp_steps": ran,
            "ramp_s": ramp_s,
            "kernel_timed_ms": max(timed_ms - flush_ms, 0.0) / args.steps,
            "flush_ms": flush_ms,
            "p50_ms": percentile(step_gpu_ms, 50),
            "p90_ms": percentile(step_gpu_ms, 90),
            "kernel_in_step_ms": sum(a.elapsed_time(b) for a, b in kern) / len(kern)}


def graph_timed(launch, reps, warm, tail=None, on_capture_fail=None, align=None):
    """Device time per launch of `launch(i)`: WARM eager launches, then REPS
    launches (+ `tail()`, e.g. the flush that ends a captured chained
    sequence) captured into one HIP graph, replayed once untimed and once
    between two HIP events on the current stream.  The replay runs the
    launches back to back on the GPU with no host enqueue in between — eagerly
    launched steps (~30 us of Python + ctypes each) are host-bound on a slow
    host core and would time the host instead (measured: 31.6 vs 29.7 us per
    chained launch on one box).  Falls back to timed eager launches if capture
    is refused.  align(): called right before the timed replay (multi-rank:
    a barrier, so no rank's timed replay waits for a peer still in its
    untimed one).  Returns (ms per launch, "graph" | "eager")."""
    import torch
    for i in range(warm):
        launch(i)
    if tail:
        tail()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    try:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for i in range(reps):
                launch(i + 1)
            if tail:
                tail()
    except Exception:   # capture refused: time eager launches
        if on_capture_fail:
            on_capture_fail()
        torch.cuda.synchronize()
        if align:
            align()
        e0.record()
        for i in range(reps):
            launch(i + 1)
        e1.record()
        if tail:
            tail()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps, "eager"
    g.replay()
    torch.cuda.synchronize()
    if align:
        align()
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps, "graph"


def kernel_pass(ep, pool, reps=200, warm=200):
    """The rollout kernel alone: REPS back-to-back launches replayed from a
    HIP graph (graph_timed), rotating over the resident batches (at least 4 x
    the batch bytes between two uses of a batch, so no launch is served from
    the 256 MiB Infinity Cache)."""
    saved = ep.cur

    def one(i):
        ep.cur = pool[i % len(pool)]
        ep.partials()
    ms, _ = graph_timed(one, reps, warm)
    ep.cur = saved
    return ms


def max_over_ranks(x, device):
    """max of a number over the ranks (x itself without a process group)."""
    import torch
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return x
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def exchange_chain_pass(ep, pool, reps=100, warm=200):
    """The exchange-form chained launch (mpc_episode_exchange_step: selection
    over step k-1's gathered candidates + episode update + rollout of step k +
    this rank's candidate) alone: per launch a pair of HIP events on the
    episode's stream around the launch only — the all_gather that follows it
    is outside the pair — averaged over REPS real steps after WARM untimed
    ones (the clock ramp, as chain_pass)."""
    import torch
    for i in range(warm):
        ep.step(controls=pool[i % len(pool)])
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(reps)]
    for i in range(reps):
        ep.step(events=evs[i], controls=pool[(i + 1) % len(pool)])
    ep.flush()
    torch.cuda.synchronize()
    return sum(a.elapsed_time(b) for a, b in evs) / reps


# the exchange form of the chained kernel (k_episode_chain<..., kChainXchg, ...>)
XCHG_KERNEL = "k_episode_chain[exchange]"
# ... and its P2P form (k_episode_chain<..., kChainP2P, ...>: the one-GPU
# chain's records + block 0's mailbox exchange)
P2P_KERNEL = "k_episode_chain[p2p]"
# committed PMC summaries (tools/pmc.sh + tools/pmc_summary.py), per kernel
# one per measured size; the one whose algorithmic bytes match is used
TRAFFIC_JSON = {"k_rollout_argmin_stream": ["r03_traffic_stream.json"],
                "k_episode_chain": ["r06_final/traffic_chain_tiled.json",
                                    "r06_final/traffic_chain_tiled_D.json",
                                    "r06_final/traffic_chain_tiled_Dtotal.json",
                                    "r04_final/close/traffic_chain.json",
                                    "r05/traffic_chain_D.json"],
                XCHG_KERNEL: ["r04/traffic_chain_xchg.json"],
                P2P_KERNEL: ["r06_final/traffic_chain_p2p_tiled.json",
                             "r04_final/close/traffic_chain_p2p.json",
                             "r05/traffic_chain_p2p_D.json",
                             "r05/traffic_chain_p2p_tiled_D.json"]}


def traffic_summary(traffic_json, kernel, bytes_launch, layout="soa"):
    """(summary dict, path) of the PMC summary measured on this kernel at this
    algorithmic size and control layout (traffic_json: an explicit file), else
    (None, None)."""
    paths = ([traffic_json] if traffic_json else
             [os.path.join(REPO, "profiles", p) for p in TRAFFIC_JSON.get(kernel, [])])
    for path in paths:
        if not path or not os.path.exists(path):
            continue
        with open(path) as fh:
            t = json.load(fh)
        if (abs(t.get("algorithmic_bytes_per_launch", -1) - bytes_launch) < 1
                and t.get("kernel", kernel) == kernel and t.get("layout", "soa") == layout):
            return t, path
    return None, None

# fp64 VALU counters (tools/pmc_valu.sh: SQ_INSTS_VALU_{FMA,ADD,MUL,TRANS}_F64,
# SQ_INSTS_VALU) of each kernel at the size it was measured on:
# (kernel, integrator) -> (summary, candidates, horizon) — config C, or the
# S1 = 451 full tree of config F (candidates = leaves)
VALU_JSON = {("k_episode_chain", "rect+cum"): ("r06_final/valu/chain.json", 1_000_000, 10),
             ("k_rollout_argmin_stream", "qk21"): ("r06_final/valu/qk21.json", 1_000_000, 10),
             ("k_rollout_generated", "rect+cum"): ("r06_final/valu/gen.json", 1_000_000, 10),
             ("k_ft_leaves", "rect+rot"): ("r06_final/valu/ft.json", 451 ** 3, 3),
             # the device-resident episode drivers: counters of the whole run,
             # keyed (episodes, max_calls) of workloads R and G as the bench runs
             # them (G: every k_ftl_* launch of the run summed)
             ("k_episodes_run", "qk21"): ("r06_final/valu/episodes_R.json", 1000, 1000),
             ("k_ftl_", "rect+rot"): ("r06_final/valu/ftepisodes_G.json", 1000, 50)}


def valu_roofline(kernel, integrator, ms, n_cand, n_steps, note=None):
    """SURVEY §8(d)'s second roofline: fp64 operations per launch from the
    committed PMC counters (64 lanes x (2 FMA + ADD + MUL + TRANS) per
    wave-instruction; inactive lanes counted, so an upper bound) over the
    measured duration, against the 78.6 TFLOP/s fp64 vector peak; and the
    VALU issue share (all VALU wave-instructions at 4 cycles on 1024 SIMDs at
    2.4 GHz).  None when no summary was measured for this kernel and size."""
    spec = VALU_JSON.get((kernel, integrator))
    if spec is None or spec[1] != n_cand or spec[2] != n_steps or not ms:
        return None
    path = os.path.join(REPO, "profiles", spec[0])
    if not os.path.exists(path):
        return None
    with open(path) as fh:
        t = json.load(fh)
    ops = t.get("fp64_ops_per_launch")
    insts = t.get("counters_median_per_launch", {}).get("SQ_INSTS_VALU")
    if not ops or t.get("kernel") != kernel:
        return None
    tf = ops / (ms * 1e-3) / 1e12
    out = {"bound": "valu-fp64", "achieved": tf, "peak": FP64_VECTOR_PEAK_TFLOPS,
           "unit": "TFLOP/s", "frac": tf / FP64_VECTOR_PEAK_TFLOPS, "kernel": kernel,
           "fp64_ops_per_launch": ops,
           "valu_issue_share": (insts * 4.0 / (1024 * 2.4e9 * ms * 1e-3)) if insts else None,
           "source": os.path.relpath(path, REPO)}
    if note:
        out["note"] = note
    return out


def chain_pass(ep, pool, reps=200, warm=200):
    """The chained launch (rollout of step k + completion of step k-1): REPS
    real steps rotating over the resident batches, captured with the flush
    that ends the sequence and replayed back to back from a HIP graph
    (graph_timed; the one flush launch is included, +~0.05 us per launch),
    after WARM eager ones (the GPU's clocks ramp over the first few hundred
    launches); the episode goes on."""
    def one(i):
        ep.step(controls=pool[i % len(pool)])

    def lost():                 # a refused capture: the captured steps never ran
        if hasattr(ep, "_pending"):
            ep._pending = None
    import torch.distributed as dist
    align = dist.barrier if dist.is_initialized() and dist.get_world_size() > 1 else None
    n0 = ep.steps_enqueued
    ms, how = graph_timed(one, reps, warm, tail=ep.flush, on_capture_fail=lost, align=align)
    # warm + 2 replays (or the eager fallback's reps) of real steps ran
    ep.steps_enqueued = n0 + warm + (2 * reps if how == "graph" else reps)
    return ms


def run_pass(ep, pool, reps=200, warm=2):
    """The persistent run sustained: ONE run of REPS steps rotating over the
    resident batches (ceil(REPS / 64) launches), captured into a HIP graph,
    replayed WARM times untimed and once between two HIP events; ms per step.
    The episode goes on."""
    import torch
    batches = [pool[i % len(pool)] for i in range(reps)]
    n0 = ep.steps_enqueued
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        ep.run(batches)
    for _ in range(warm):
        g.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    ep.steps_enqueued = n0 + (warm + 1) * reps
    return e0.elapsed_time(e1) / reps


def roofline(achieved, bytes_launch, traffic_json, kernel="k_rollout_argmin_stream",
             layout="soa"):
    """traffic: HBM bytes per launch from the committed PMC summary, used only
    when it was measured on the same kernel, algorithmic size and layout."""
    traffic, src = None, None
    t, path = traffic_summary(traffic_json, kernel, bytes_launch, layout)
    if t:
        traffic, src = t.get("hbm_bytes_per_launch"), os.path.relpath(path, REPO)
    return {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": src,
            "kernel": kernel, "layout": layout, "algorithmic_bytes_per_launch": bytes_launch}


def bench_robots(args, wl, eng, rank, world, cpu):
    """Config E: robots sharded over ranks, one batched launch per step."""
    import numpy as np
    import torch
    import torch.distributed as dist
    from diplomjourney_amd import math_model_tree as mmt
    from diplomjourney_amd.abi import make_problem, PROBLEM_BYTES
    from diplomjourney_amd.distributed import shard_range
    from diplomjourney_amd.episode import percentile
    from diplomjourney_amd.expansion import problems_to_device, results_from_device
    R_total, cand, n_steps = wl["robots"], wl["cand"], wl["n_steps"]
    lo, hi = shard_range(R_total, rank, world)
    R = hi - lo
    probs = []
    for r in range(lo, hi):
        g = np.random.default_rng(20261015 + r)              # PCG64 per robot
        x0, y0 = g.uniform(-10, 10, 2)
        phi0 = g.uniform(-math.pi, math.pi)
        xt, yt = g.uniform(x0 - 10, x0 + 10), g.uniform(y0 - 10, y0 + 10)
        probs.append(make_problem(x0, y0, phi0, xt, yt, x0, y0, mmt.L, 0.05, 0.1))
    V = torch.tensor(mmt.vector_of_velocities(0.5), dtype=torch.float64, device=eng.device)
    B = torch.tensor(mmt.vector_of_beta_angles(0.0), dtype=torch.float64, device=eng.device)
    v = torch.empty((n_steps, R * cand), dtype=torch.float64, device=eng.device)
    b = torch.empty_like(v)
    for i in range(R):
        eng.sample_controls(V, B, cand, n_steps, 20261015 + lo + i, v_out=v[:, i * cand:],
                            beta_out=b[:, i * cand:], ld=R * cand)
    probs_dev = problems_to_device(probs, eng.device)
    out = torch.zeros(R * eng.result.numel(), dtype=torch.uint8, device=eng.device)
    host = torch.empty(out.numel(), dtype=torch.uint8).pin_memory()
    step_ms, kern = [], []
    state = torch.empty((R, 3), dtype=torch.float64)

    def one(timed):
        t0 = time.perf_counter()
        if timed:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        eng.rollout_argmin_batched(probs_dev, v, b, cand, integrator=args.integrator, out=out)
        if timed:
            e1.record()
        host.copy_(out, non_blocking=True)
        torch.cuda.current_stream().synchronize()
        if timed:
            kern.append(e0.elapsed_time(e1))
        step_ms.append((time.perf_counter() - t0) * 1e3)

    for _ in range(args.warmup):
        one(False)
    step_ms.clear()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=eng.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    res = results_from_device(out)
    assert all(r.index >= 0 for r in res)
    kern_ms = sum(kern) / len(kern)
    bytes_launch = 16.0 * n_steps * R * cand
    outd = {
        "metric": METRIC, "value": R_total * cand * args.steps / elapsed, "unit": "rollouts/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": wl["desc"], "n_steps": n_steps, "robots_per_gpu": R,
                   "candidates_per_robot": cand, "integrator": args.integrator,
                   "parallelism": f"robot-sharded x{world}, no exchange"},
        "p50_ms": percentile(step_ms, 50), "kernel_ms": kern_ms,
        # kern_ms brackets both launches of the call (the rollout and the
        # per-robot finalize, ~7 us of it)
        "roofline": roofline(bytes_launch / (kern_ms * 1e-3) / 1e9, bytes_launch,
                             args.traffic_json,
                             kernel="k_rollout_argmin_batched+k_finalize_batched"),
        "cpu_baseline": cpu,
    }
    if rank == 0:
        print(json.dumps(outd), flush=True)
    if world > 1:
        dist.destroy_process_group()


def bench_fulltree(args, wl, eng, rank, world, cpu):
    """Config F: the run_math_model full tree; one mpc_fulltree_argmin per MPC
    step inside the drop-in's episode (host reads the 200-B result each step,
    as predictive_control returns it).  G > 1: the leaves of every step are
    sharded over the ranks (contiguous work-item ranges) and one all_gather of
    the 200-B results selects the winner on every rank: strong scaling."""
    import math as _m
    import torch
    import torch.distributed as dist
    from diplomjourney_amd import run_math_model as rmm
    from diplomjourney_amd.episode import percentile
    rmm.INTEGRATOR = args.integrator
    rmm.configure(0.1, _m.radians(3))
    if world > 1:
        rmm.shard_over(dist.group.WORLD)
    s1 = int(rmm.size_max_1)
    leaves = s1 ** 3
    rmm.start_episode(-3.0, -2.0, 0.3, 4.0, 5.0)

    trace = []

    def step():
        c = rmm.predictive_control(rmm.x, rmm.y, rmm.phi, rmm.v, rmm.x_t, rmm.y_t)
        rmm.x, rmm.y, rmm.phi, rmm.v, rmm.beta = c
        trace.append([float(z) for z in c] + [float(rmm.optimal_criterion)])

    for _ in range(args.warmup):
        step()
    ms = []
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        a = time.perf_counter()
        step()
        ms.append((time.perf_counter() - a) * 1e3)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=eng.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    per_step = elapsed / args.steps
    if args.dump_log and rank == 0:
        with open(args.dump_log, "w") as fh:
            json.dump(trace, fh)
    # The launches alone (mpc_fulltree_argmin: control table, leaves, selection)
    # on the episode's last problem, back to back between HIP events on the
    # current stream: the duration the rooflines divide by (the step above
    # adds the drop-in's host work and the 200-B read-back).
    from diplomjourney_amd.abi import MpcFulltreeProblem
    from diplomjourney_amd.expansion import fulltree_argmin
    feng, (fvg, fbg) = rmm._device()
    fp = MpcFulltreeProblem(float(rmm.x), float(rmm.y), float(rmm.phi), float(rmm.x_t),
                            float(rmm.y_t), float(rmm.x_0), float(rmm.y_0),
                            float(_m.atan(rmm.x_t / rmm.y_t)), float(rmm.L), float(rmm.t),
                            float(rmm.t + rmm.delta_t))
    shard = (dist.get_rank(), world) if world > 1 else (0, 1)
    for _ in range(3):
        fulltree_argmin(feng, fp, fvg, fbg, float("inf"), args.integrator, *shard)
    reps = 20
    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    ev[0].record()
    for _ in range(reps):
        fulltree_argmin(feng, fp, fvg, fbg, float("inf"), args.integrator, *shard)
    ev[1].record()
    torch.cuda.synchronize()
    launch_ms = ev[0].elapsed_time(ev[1]) / reps
    flops = FT_FLOPS_PER_LEAF[args.integrator] * leaves / world / (launch_ms * 1e-3)   # per GPU
    out = {
        "metric": METRIC, "value": leaves * args.steps / elapsed, "unit": "leaves/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": per_step * 1e3, "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": wl["desc"], "s1": s1, "leaves_per_step": leaves,
                   "integrator": args.integrator,
                   "parallelism": (f"leaf-sharded x{world}, all_gather(200 B)/step"
                                   if world > 1 else "single GPU")},
        "p50_ms": percentile(ms, 50),
        "launch_ms": launch_ms,
        "launch_note": "mpc_fulltree_argmin's three launches (k_ft_leaves ~96%), HIP events "
                       "around 20 back-to-back calls on the last step's problem",
        "roofline": {"bound": "valu-fp64", "achieved": flops / 1e12,
                     "peak": FP64_VECTOR_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": flops / 1e12 / FP64_VECTOR_PEAK_TFLOPS, "traffic": None,
                     "kernel": "k_ft_leaves",
                     "note": "algorithmic fp64 ops per leaf as written (FT_FLOPS_PER_LEAF) over "
                             "launch_ms; leaves are generated from the index, no HBM stream"},
        "roofline_valu": valu_roofline("k_ft_leaves", args.integrator, launch_ms * world,
                                       leaves, 3,
                                       note="counted fp64 ops of one MPC step (all leaves, PMC) "
                                            "over launch_ms x ranks"),
        "cpu_baseline": cpu,
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def bench_tree_episodes(args, wl, eng, rank, world, cpu):
    """The named entry: run_math_model.py's seeded episode loop
    for 1000 episodes, its MPC step the tree expansion (Fact 2), robots
    sharded over ranks (no exchange), device-resident (episode.DeviceEpisodes:
    one block per robot runs its episode's MPC steps back to back — grid,
    enumeration, expansion, winner, update — in ONE launch).  Timed: the
    launch of up to K = --steps MPC steps of every episode (K caps an
    episode's calls; the log of every step is written) between syncs;
    ms_per_step = that time / the longest episode's calls (a lockstep-
    equivalent step of all running episodes)."""
    import torch
    import torch.distributed as dist
    from diplomjourney_amd import run_math_model as rmm
    from diplomjourney_amd.abi import MPC_EP_ARRIVED, MPC_EP_BREAK
    from diplomjourney_amd.distributed import shard_range
    from diplomjourney_amd.episode import DeviceEpisodes, tree_episode_config
    starts = rmm.draw_starts(wl["robots"], seed=20261015)
    lo, hi = shard_range(len(starts), rank, world)
    cfgs = [tree_episode_config(s, args.steps) for s in starts[lo:hi]]
    eps = DeviceEpisodes(eng, cfgs, 3, args.integrator, log_capacity=args.steps)
    for _ in range(max(1, args.warmup)):                # warmup: whole runs
        eps.reset()
        eps.run(args.steps)
    eps.reset()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eps.run(args.steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    calls, stop, cands = eps.read_progress()
    t = torch.tensor([elapsed, float(calls.sum()), float(cands.sum()), float(calls.max())],
                     dtype=torch.float64, device=eng.device)
    if world > 1:
        mx = t[[0, 3]].clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        t[0], t[3] = mx[0], mx[1]
    elapsed, n_calls, n_cands, lockstep = (float(t[0]), int(t[1]), int(t[2]), int(t[3]))
    stops = {}
    for st in stop:
        k = ("recursive_error" if st & MPC_EP_BREAK else
             "on_target" if st & MPC_EP_ARRIVED else "max_calls")
        stops[k] = stops.get(k, 0) + 1
    out = {
        "metric": METRIC, "value": n_cands / elapsed, "unit": "rollouts/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / max(1, lockstep) * 1e3,
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (the script's seeded start/target draws)",
        "config": {"workload": wl["desc"], "n_steps": 3, "episodes": wl["robots"],
                   "mpc_calls": n_calls, "lockstep_steps": lockstep,
                   "integrator": args.integrator, "episode_stops_rank0": stops,
                   "episode_loop": "device-resident: one block per robot, one launch for all "
                                   "steps (mpc_episodes_run)",
                   "parallelism": f"robot-sharded x{world}, no exchange"},
        "episodes_per_s": wl["robots"] / elapsed,
        "p50_ms": None,
        "p50_note": "ms_per_step = the run's time / the longest episode's MPC calls",
        "roofline": None,
        "roofline_valu": valu_roofline("k_episodes_run", args.integrator, elapsed * 1e3,
                                       wl["robots"], args.steps,
                                       note="counted fp64 ops of the whole one-launch run "
                                            "(PMC, tools/prof_kernel.py tree_episodes) over the "
                                            "timed run; the candidates never touch HBM, so "
                                            "the fp64 VALU is the bound"),
        "cpu_baseline": cpu,
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def bench_episodes(args, wl, eng, rank, world, cpu):
    """Config G: the script's episode loop for 1000 episodes at once (robots
    sharded over ranks, no exchange), device-resident (run_batched ->
    mpc_fulltree_episodes_run, csrc/mpc_ftepisodes.h: per call three launches
    over the robots still running — stop rules + compaction + the call's
    control table, the leaves of every live robot spread over the whole GPU,
    one update block per live robot; no host step).  Timed: up to K = --steps
    calls of every episode (K as max_calls) between syncs; ms_per_step = that
    time / the longest episode's calls (a lockstep-equivalent step)."""
    import math as _m
    import torch
    import torch.distributed as dist
    from diplomjourney_amd import run_math_model as rmm
    from diplomjourney_amd.distributed import shard_range
    rmm.INTEGRATOR = args.integrator
    rmm.configure(0.25, _m.radians(10))
    s1 = int(rmm.size_max_1)
    starts = rmm.draw_starts(wl["robots"], seed=20261015)
    lo, hi = shard_range(len(starts), rank, world)
    from diplomjourney_amd.abi import MPC_EP_ARRIVED, MPC_EP_BREAK
    eps_dev = rmm.device_ft_episodes(starts[lo:hi], args.steps, args.integrator,
                                     log_capacity=args.steps)
    for _ in range(max(1, args.warmup // 20)):                           # warmup: whole runs
        eps_dev.reset()
        eps_dev.run(args.steps)
    eps_dev.reset()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eps_dev.run(args.steps)                  # ONE launch: every call of every episode
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    calls, stop, _ = eps_dev.read_progress()
    outs = [(None, "recursive_error" if st & MPC_EP_BREAK else
             "on_target" if st & MPC_EP_ARRIVED else "max_calls") for st in stop]
    robot_steps = int(calls.sum())
    t = torch.tensor([elapsed, robot_steps, int(calls.max())], dtype=torch.float64,
                     device=eng.device)
    if world > 1:
        mx = t[[0, 2]].clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        t[0], t[2] = mx[0], mx[1]
    elapsed, robot_steps, lockstep = float(t[0]), float(t[1]), int(t[2])
    leaves = robot_steps * s1 ** 3
    stops = {}
    for _, st in outs:
        stops[st] = stops.get(st, 0) + 1
    flops = FT_FLOPS_PER_LEAF[args.integrator] * leaves / world / elapsed      # per GPU
    out = {
        "metric": METRIC, "value": leaves / elapsed, "unit": "leaves/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / max(1, lockstep) * 1e3,
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (the script's seeded start/target draws)",
        "config": {"workload": wl["desc"], "s1": s1, "robots": wl["robots"],
                   "robot_steps": robot_steps, "lockstep_steps": lockstep,
                   "integrator": args.integrator, "episode_stops_rank0": stops,
                   "episode_loop": "device-resident lockstep over the live robots: per call "
                                   "k_ftl_prepare + k_ftl_leaves (grid spread over the live "
                                   "robots) + k_ftl_update (mpc_fulltree_episodes_run)",
                   "parallelism": f"robot-sharded x{world}, no exchange"},
        "p50_note": "ms_per_step = the run's time (one launch + sync) / the longest "
                    "episode's calls",
        "roofline": {"bound": "valu-fp64", "achieved": flops / 1e12,
                     "peak": FP64_VECTOR_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": flops / 1e12 / FP64_VECTOR_PEAK_TFLOPS, "traffic": None,
                     "kernel": "k_ftl_leaves",
                     "note": "algorithmic fp64 ops per leaf as written (FT_FLOPS_PER_LEAF) x "
                             "the leaves scored, over the whole timed run"},
        "roofline_valu": valu_roofline("k_ftl_", args.integrator, elapsed * 1e3,
                                       wl["robots"], args.steps,
                                       note="counted fp64 ops of the whole run (PMC) over the "
                                            "timed run"),
        "cpu_baseline": cpu,
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
