"""Isolated timing of vaesne_linear_bwd_weight at the step's large-M shapes (the output
head's fc1, a decoder in_proj, an FFN layer): HIP events around 50 launches each.
    VAESNE_HIP_LIB=<lib> python tools/ab/wgrad_ab.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "vaesne-dev_amd"))
from VAESNe._lib import lib  # noqa: E402

dev = torch.device("cuda", 0)
M = 8 * 32 * 982
for (O, I, x2, act) in [(32, 32, True, 0), (96, 32, False, 0), (32, 32, False, 0), (32, 32, False, 2)]:
    dy = torch.randn(M, O, device=dev)
    x = torch.randn(M, I, device=dev)
    xx = torch.randn(M, I, device=dev) if x2 else None
    z = torch.randn(M, O, device=dev) if act else None
    dW = torch.empty(O, I, device=dev)
    db = torch.empty(O, device=dev)
    ws = torch.empty(lib.linear_bwd_weight_workspace(M, O, I) // 4 + 1, device=dev)
    s = torch.cuda.current_stream().cuda_stream

    def run():
        lib.linear_bwd_weight(dy.data_ptr(), O, z.data_ptr() if act else None, O, act,
                              x.data_ptr(), I, xx.data_ptr() if x2 else None, I, M, O, I,
                              dW.data_ptr(), db.data_ptr(), 0, ws.data_ptr(), None, s)
    for _ in range(5):
        run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        run()
    e1.record()
    torch.cuda.synchronize()
    print(f"O={O} I={I} x2={x2} act={act}: {e0.elapsed_time(e1) / 50 * 1e3:.1f} us")
