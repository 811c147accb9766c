"""Do independent branches of a captured hipGraph run concurrently?  Two chains
of N tiny dependent kernels on two streams inside one capture, vs one chain of
N, vs one chain of 2N; replay time per graph.
    python profiles/graph_branch_probe.py"""
import time

import torch


def chain(x, n):
    for _ in range(n):
        x.mul_(1.0001).add_(1e-4)
    return x


def timed(g, reps=50):
    g.replay()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def main():
    dev = torch.device("cuda:0")
    n = 100
    a = torch.zeros(256, device=dev)
    b = torch.zeros(256, device=dev)
    side = torch.cuda.Stream(dev)
    res = {}
    for name in ("one", "two_serial", "two_streams", "two_streams_interleaved"):
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            with torch.cuda.graph(g):
                main = torch.cuda.current_stream()
                if name == "one":
                    chain(a, n)
                elif name == "two_serial":
                    chain(a, n)
                    chain(b, n)
                elif name == "two_streams":
                    side.wait_stream(main)
                    with torch.cuda.stream(side):
                        chain(b, n)
                    chain(a, n)
                    main.wait_stream(side)
                else:
                    side.wait_stream(main)
                    for _ in range(n):
                        with torch.cuda.stream(side):
                            chain(b, 1)
                        chain(a, 1)
                    main.wait_stream(side)
        res[name] = timed(g)
    print({k: round(v, 3) for k, v in res.items()}, "ms per replay (2 kernels per chain link)")


if __name__ == "__main__":
    main()
