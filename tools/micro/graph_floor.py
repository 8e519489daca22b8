"""Per-node time of a replayed hipGraph of back-to-back dependent kernels that
do (almost) nothing: the floor under a latency-bound chained step (config B).
    python tools/micro/graph_floor.py"""
import torch


def per_node(fn, n=500, reps=5):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b) / n * 1e3)
    return best


x1 = torch.zeros(1, device="cuda")
x2 = torch.zeros(197 * 256, device="cuda")
x3 = torch.zeros(1536 * 256, device="cuda")
print("graph node, 1 block       : %.2f us" % per_node(lambda: x1.add_(1)))
print("graph node, 197 blocks    : %.2f us" % per_node(lambda: x2.add_(1)))
print("graph node, 1536 blocks   : %.2f us" % per_node(lambda: x3.add_(1)))
