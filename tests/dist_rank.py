"""One rank of tests/test_gpu_parity.py::test_exchange_chain_two_ranks_on_one_gpu
(started as a child process per rank; gloo stages the exchange through host
memory, so several ranks can share one GPU).  Writes its episode log as JSON.
    python tests/dist_rank.py RANK WORLD PORT N_TOTAL N_STEPS STEPS OUT.json [gather|p2p] [DELAY_S]
(gather: the all_gather of the candidates, staged through the host by gloo;
p2p: the mailboxes, IPC handles exchanged over gloo once.  DELAY_S: rank 1
holds its stream back that long (a spinning kernel) before its 10th step, so
its peers' launches wait for its candidate — a lagging rank)"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    rank, world, port, n_total, ns, steps = (int(a) for a in sys.argv[1:7])
    out = sys.argv[7]
    mode = sys.argv[8] if len(sys.argv) > 8 else "gather"
    delay_s = float(sys.argv[9]) if len(sys.argv) > 9 else 0.0
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
    import time
    t0 = time.perf_counter()

    def note(msg):
        print(f"[rank {rank} +{time.perf_counter() - t0:.3f}s] {msg}", file=sys.stderr, flush=True)

    held = None
    rate = None
    if delay_s > 0 and rank == 1:   # spin cycles per ms of torch.cuda._sleep, measured
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
        torch.cuda._sleep(100_000_000)           # ~40 ms: launch overhead negligible
        ev[1].record()
        torch.cuda.synchronize()
        rate = 100_000_000 / max(ev[0].elapsed_time(ev[1]), 1e-3)
        note(f"_sleep: {rate:.0f} cycles/ms")
    for i in range(steps):
        if delay_s > 0 and rank == 1 and i == 10:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
            torch.cuda._sleep(int(delay_s * 1e3 * rate))
            ev[1].record()
            held = ev
        ep.step(controls=pool[i % 4])
        if i % 10 == 9:
            note(f"enqueued {i + 1} steps")
    ep.flush()
    note("flushed; reading the log")
    log = [[r.step, r.index, r.cost, r.x, r.y, r.phi, r.v, r.beta, r.p, r.episode, r.status]
           for r in ep.read_log()]
    err = ep.chain_error()
    note(f"log read, chain_error {err}")
    with open(out, "w") as fh:
        json.dump({"log": log, "chain_error": err, "winner": ep.winner.cpu().tolist(),
                   "held_ms": held[0].elapsed_time(held[1]) if held else 0.0}, fh)
    if mode == "p2p":
        dist.barrier()          # no peer still stores into this rank's mailbox
        ep.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
