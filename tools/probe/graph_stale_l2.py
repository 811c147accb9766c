"""Probe (not product): can a captured hipGraph's kernel on one stream read an L2 line
that another stream's kernel made stale?  Per replay: side reads X (caching it), main
then rewrites X, side reads X again after waiting on main: the second read must see the
new values."""
import os
import torch

N = int(os.environ.get("N", str(1 << 18)))
R = int(os.environ.get("R", "300"))
side = torch.cuda.Stream()
inp = torch.zeros(N, device="cuda")
X = torch.zeros(N, device="cuda")
y1 = torch.empty(N, device="cuda")
y2 = torch.empty(N, device="cuda")
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    cap = torch.cuda.current_stream()
    side.wait_stream(cap)
    with torch.cuda.stream(side):
        torch.mul(X, 1.0, out=y1)
    cap.wait_stream(side)
    X.copy_(inp)
    side.wait_stream(cap)
    with torch.cuda.stream(side):
        torch.mul(X, 1.0, out=y2)
    cap.wait_stream(side)
bad = 0
for i in range(R):
    inp.fill_(float(i + 1))
    g.replay()
    torch.cuda.synchronize()
    if not bool((y2 == float(i + 1)).all()):
        bad += 1
        if bad <= 5:
            print("replay", i, "stale values:", torch.unique(y2)[:4].tolist())
print(f"{bad} of {R} replays read stale data")
