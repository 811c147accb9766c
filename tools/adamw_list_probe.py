"""One torch.optim.AdamW step vs vaesne_adamw_list on one tensor: mismatch counts of
p, exp_avg, exp_avg_sq per contraction variant (debug aid for VAESNe._update)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "vaesne-dev_amd"))
from VAESNe import _update  # noqa: E402


def run(dev_update, fma, steps):
    g = torch.Generator().manual_seed(0)
    p = torch.nn.Parameter((torch.randn(4096, generator=g)).cuda())
    opt = torch.optim.AdamW([p], lr=1e-2)
    upd = _update.TorchAdamWUpdater(opt)
    _update.TORCH_FMA = fma
    for s in range(steps):
        p.grad = (torch.randn(4096, generator=g) * 1e-2).cuda()
        if dev_update:
            assert upd.ready()
            upd.update(None)
        else:
            opt.step()
    torch.cuda.synchronize()
    st = opt.state[p]
    return p.detach().clone(), st["exp_avg"].clone(), st["exp_avg_sq"].clone()


for steps in (1, 2, 3):
    ref = run(False, 1, steps)
    for fma in (1, 0):
        got = run(True, fma, steps)
        print(steps, fma, [int((a != b).sum()) for a, b in zip(got, ref)],
              [float((a - b).abs().max()) for a, b in zip(got, ref)])
