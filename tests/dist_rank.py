"""One rank of tests/test_gpu_parity.py::test_exchange_chain_two_ranks_on_one_gpu
(started as a child process per rank; gloo stages the exchange through host
memory, so several ranks can share one GPU).  Writes its episode log as JSON.
    python tests/dist_rank.py RANK WORLD PORT N_TOTAL N_STEPS STEPS OUT.json [gather|p2p]
(gather: the all_gather of the candidates, staged through the host by gloo;
p2p: the mailboxes, IPC handles exchanged over gloo once)"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    rank, world, port, n_total, ns, steps = (int(a) for a in sys.argv[1:7])
    out = sys.argv[7]
    mode = sys.argv[8] if len(sys.argv) > 8 else "gather"
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    from diplomjourney_amd import math_model_tree as mmt
    from diplomjourney_amd.episode import DeviceEpisode
    from diplomjourney_amd.expansion import Expansion
    eng = Expansion("cuda:0")
    ep = DeviceEpisode(eng, n_total, ns, rank=rank, world=world, integrator="rect+cum",
                       exchange=True, chain=True, log_capacity=256, max_steps=40,
                       p2p=mode == "p2p")
    V = torch.tensor(mmt.vector_of_velocities(0.5), dtype=torch.float64, device="cuda")
    B = torch.tensor(mmt.vector_of_beta_angles(0.0), dtype=torch.float64, device="cuda")
    pool = [eng.sample_controls(V, B, ep.n_local, ns, 4100 + i, index_base=ep.lo)
            for i in range(4)]
    for i in range(steps):
        ep.step(controls=pool[i % 4])
    ep.flush()
    log = [[r.step, r.index, r.cost, r.x, r.y, r.phi, r.v, r.beta, r.p, r.episode, r.status]
           for r in ep.read_log()]
    err = ep.chain_error()
    with open(out, "w") as fh:
        json.dump({"log": log, "chain_error": err, "winner": ep.winner.cpu().tolist()}, fh)
    if mode == "p2p":
        dist.barrier()          # no peer still stores into this rank's mailbox
        ep.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
