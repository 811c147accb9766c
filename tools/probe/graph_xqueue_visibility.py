"""Probe (not product): memory visibility across the streams of a captured hipGraph.
Side-stream kernels write buffers that main-stream kernels read after the join (and the
reverse inside the fork); the input changes before every replay, so a consumer that sees
the previous replay's data shows up as a mismatch."""
import os
import torch

N = int(os.environ.get("N", str(1 << 16)))
R = int(os.environ.get("R", "300"))
main = torch.cuda.current_stream()
side = torch.cuda.Stream()
inp = torch.zeros(N, device="cuda")
bufs = [torch.empty(N, device="cuda") for _ in range(8)]
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    cap = torch.cuda.current_stream()
    a = inp * 1.0                       # main
    side.wait_stream(cap)
    with torch.cuda.stream(side):
        torch.mul(a, 2.0, out=bufs[0])     # side reads main's a, writes b0
        torch.add(bufs[0], 1.0, out=bufs[1])
    cap.wait_stream(side)
    torch.add(bufs[1], 3.0, out=bufs[2])   # main reads side's b1
    side.wait_stream(cap)
    with torch.cuda.stream(side):
        torch.mul(bufs[2], 0.5, out=bufs[3])
    torch.mul(bufs[2], 0.25, out=bufs[4])  # main, beside side
    cap.wait_stream(side)
    out = bufs[3] + bufs[4]
bad = 0
for i in range(R):
    inp.fill_(float(i))
    g.replay()
    torch.cuda.synchronize()
    exp = ((2.0 * i + 1.0) + 3.0) * 0.75
    err = (out - exp).abs().max().item()
    if err > 1e-3:
        bad += 1
        if bad <= 5:
            print("replay", i, "max err", err, "unique", torch.unique(out)[:4].tolist())
print(f"{bad} of {R} replays read stale data")
