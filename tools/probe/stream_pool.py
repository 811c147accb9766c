"""Probe (not product): handles of consecutively created torch.cuda.Stream objects."""
import torch
s = [torch.cuda.Stream() for _ in range(6)]
print([hex(x.cuda_stream) for x in s])
print("default", hex(torch.cuda.default_stream().cuda_stream), "current", hex(torch.cuda.current_stream().cuda_stream))
