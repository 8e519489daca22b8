"""Minimal driver for rocprofv3 counter passes: sample B distinct candidate
batches, then launch only the rollout kernel `reps` times rotating over them
(B x batch bytes between two uses of a batch > 256 MiB Infinity Cache, so the
launches stream from HBM as in the bench).
    python tools/prof_kernel.py [n_cand] [n_steps] [integ] [reps] [batches]
integ "chain": chained rect+cum episode steps instead (mpc_episode_chain_step,
the bench default's launch: rollout of step k + completion of step k-1);
"xchg": the exchange form of the chained step (mpc_episode_exchange_step +
the RCCL all_gather, over a 1-rank nccl group: the N > 1 bench's launch);
"p2p": the collective-free exchange form (mpc_episode_p2p_step, one rank: the
N > 1 bench's launch); chain / p2p with MPC_LAYOUT=tiled in the environment:
tiled batches (MPC_LAYOUT_TILED, the bench's default);
"generated": generated-controls episode steps (k_rollout_generated, rect+cum);
"fulltree": config F's full-tree MPC steps (k_ft_leaves, S1 = 451, n_cand and
n_steps ignored);
"tree_episodes" / "ft_episodes": workload R / G's one-launch episode runs
(n_cand = episodes, n_steps = max_calls)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from diplomjourney_amd import math_model_tree as mmt  # noqa: E402
from diplomjourney_amd.abi import make_problem  # noqa: E402
from diplomjourney_amd.expansion import Expansion  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    ns = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    integ = sys.argv[3] if len(sys.argv) > 3 else "rect+rot"
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
    nb = int(sys.argv[5]) if len(sys.argv) > 5 else 4
    eng = Expansion("cuda:0")
    if integ == "fulltree":
        import math
        from diplomjourney_amd import run_math_model as rmm
        rmm.INTEGRATOR = "rect+rot"
        rmm.configure(0.1, math.radians(3))
        rmm.start_episode(-3.0, -2.0, 0.3, 4.0, 5.0)
        for _ in range(reps):
            c = rmm.predictive_control(rmm.x, rmm.y, rmm.phi, rmm.v, rmm.x_t, rmm.y_t)
            rmm.x, rmm.y, rmm.phi, rmm.v, rmm.beta = c
        torch.cuda.synchronize()
        print("done fulltree", reps)
        return
    if integ in ("tree_episodes", "ft_episodes"):
        # workload R / G as bench.py runs them: n = episodes, ns = max_calls
        from diplomjourney_amd import run_math_model as rmm
        starts = rmm.draw_starts(n, seed=20261015)
        for _ in range(reps):
            if integ == "tree_episodes":
                from diplomjourney_amd.episode import DeviceEpisodes, tree_episode_config
                eps = DeviceEpisodes(eng, [tree_episode_config(s, ns) for s in starts], 3, "qk21",
                                     log_capacity=ns)
                eps.run(ns)
            else:
                import math
                rmm.INTEGRATOR = "rect+rot"
                rmm.configure(0.25, math.radians(10))
                rmm.run_batched(starts, max_calls=ns)
        torch.cuda.synchronize()
        print("done", integ, n, ns, reps)
        return
    if integ == "generated":
        from diplomjourney_amd.episode import DeviceEpisode
        ep = DeviceEpisode(eng, n, ns, integrator="rect+cum", generate=True, log_capacity=8192)
        for i in range(reps):
            ep.step()
        torch.cuda.synchronize()
        print("done generated", n, ns, reps)
        return
    V = torch.tensor(mmt.vector_of_velocities(0.5), dtype=torch.float64, device="cuda")
    B = torch.tensor(mmt.vector_of_beta_angles(0.0), dtype=torch.float64, device="cuda")
    pool = [eng.sample_controls(V, B, n, ns, 7 + i) for i in range(nb)]
    if integ in ("chain", "p2p") and os.environ.get("MPC_LAYOUT") == "tiled":
        # the bench's resident layout of the chained steps (MPC_LAYOUT_TILED)
        pool = [eng.sample_controls_tiled(V, B, n, ns, 7 + i) for i in range(nb)]
    if integ in ("chain", "xchg", "p2p"):
        from diplomjourney_amd.episode import DeviceEpisode
        xchg = integ == "xchg"
        if xchg:
            import socket
            import torch.distributed as dist
            with socket.socket() as s:
                s.bind(("127.0.0.1", 0))
                port = s.getsockname()[1]
            dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0,
                                    world_size=1, device_id=torch.device("cuda", 0))
        p2p = integ == "p2p"
        ep = DeviceEpisode(eng, n, ns, integrator="rect+cum", chain=True, exchange=xchg or p2p,
                           log_capacity=8192, p2p=p2p)
        for i in range(reps):
            ep.step(controls=pool[i % nb])
        ep.flush()
        if xchg:
            torch.cuda.synchronize()
            dist.destroy_process_group()
    else:
        prob = make_problem(0.0, 0.0, 0.3, 2, 3, 0, 0, 0.5, 0.05, 0.1)
        for i in range(reps):
            eng.partials(prob, *pool[i % nb], integ)
    torch.cuda.synchronize()
    print("done", n, ns, integ, reps, nb)


if __name__ == "__main__":
    main()
