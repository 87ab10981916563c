"""Cost of a fork / join between two streams inside a captured hipGraph (the concurrent single-GPU schedule forks the
FC weight gradient onto an aux stream after the head and joins it at the next step's head; the kernel trace shows
~5 us idle before conv_bwd and before the next head).  Tiny kernels, per-iteration replay time of:
  serial : A -> B -> C -> D on one stream
  fork   : A -> {B on aux} ; C on main ; D on main after joining aux
  fork_late : the join one kernel later (D waits for nothing, the next A waits for aux)
Usage: python scripts/diag/fork_join.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

dev = torch.device("cuda", 0)
x = [torch.zeros(1024, device=dev) for _ in range(4)]
main, aux = torch.cuda.Stream(), torch.cuda.Stream()
ITERS = 10


def body(kind):
    for _ in range(ITERS):
        if kind == "serial":
            for t in x:
                t.add_(1)
        elif kind == "fork":
            x[0].add_(1)
            aux.wait_stream(main)
            with torch.cuda.stream(aux):
                x[1].add_(1)
            x[2].add_(1)
            main.wait_stream(aux)
            x[3].add_(1)
        elif kind == "fork_late":
            x[0].add_(1)
            aux.wait_stream(main)
            with torch.cuda.stream(aux):
                x[1].add_(1)
            x[2].add_(1)
            x[3].add_(1)
            main.wait_stream(aux)


res = {}
for kind in ("serial", "fork", "fork_late"):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(main):
        body(kind)  # warm
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=main):
            body(kind)
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(7):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1000 / (20 * ITERS))
    ts.sort()
    res[kind] = ts[len(ts) // 2]
    print(f"{kind:10s} {res[kind]:7.2f} us per iteration (4 kernels)", flush=True)
print(f"fork + join cost: {res['fork'] - res['serial']:.2f} us; late join: {res['fork_late'] - res['serial']:.2f} us")
