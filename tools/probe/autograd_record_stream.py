"""Probe (not product): does autograd record a gradient produced on one stream for the
consumer node's stream?  f's backward runs on `side` and reads the gradient g's backward
produced on the main stream; right after backward() the main stream asks for a block of
the same size: the same pointer means the block went back to the pool unrecorded."""
import torch

side = torch.cuda.Stream()
PTR = []


class F(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return x * 2

    @staticmethod
    def backward(ctx, dy):
        PTR.append((dy.data_ptr(), torch.cuda.current_stream().cuda_stream))
        torch.cuda._sleep(50_000_000)      # keep the side stream busy
        return dy * 2


class G(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y):
        return y * 3

    @staticmethod
    def backward(ctx, dz):
        out = dz * 3
        PTR.append((out.data_ptr(), torch.cuda.current_stream().cuda_stream))
        return out


n = 1 << 20
x = torch.randn(n, device="cuda", requires_grad=True)
torch.cuda.synchronize()
side.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(side):
    y = F.apply(x)
torch.cuda.current_stream().wait_stream(side)
y.record_stream(torch.cuda.current_stream())
z = G.apply(y)
z.sum().backward()
t = torch.empty(n, device="cuda")
print("G.backward output on stream", PTR[1][1], "ptr", hex(PTR[1][0]))
print("F.backward read dy on stream", PTR[0][1], "ptr", hex(PTR[0][0]))
print("fresh main-stream block", hex(t.data_ptr()),
      "-> REUSED while side may still read it" if t.data_ptr() == PTR[0][0] else "-> not reused")
torch.cuda.synchronize()
