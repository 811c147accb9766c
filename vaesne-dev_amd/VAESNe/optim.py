"""FusedAdamW: torch.optim.AdamW arithmetic (the cannon scripts' optimizer,
e.g. cannon/test_photospectra.py:133, cannon/ZTF_photospect.py:119) over one
flat fp32 parameter buffer on the device.

* Parameters are re-bound as views into one flat buffer (module identity and
  state_dict keys unchanged), so the update is ONE HIP kernel launch and the
  gradient is ONE flat buffer — the unit the data-parallel all-reduce moves.
* The step counter lives on the device, so a whole training step (forward,
  backward, pack, all-reduce, update) can be captured in one hipGraph.
* Parameters whose .grad is None are skipped, as torch.optim.AdamW does.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib
from ._lib import lib, stream


class FusedAdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2,
                 grad_hook=None):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self.grad_hook = grad_hook          # callable(flat_grad) run after packing (all-reduce)
        self._flat = []
        for group in self.param_groups:
            ps = [p for p in group["params"] if p.requires_grad]
            if not ps:
                self._flat.append(None)
                continue
            dev = ps[0].device
            _lib.require_device(*ps)
            n = sum(p.numel() for p in ps)
            flat = torch.empty(n, dtype=torch.float32, device=dev)
            offs, ns = [], []
            o = 0
            with torch.no_grad():
                for p in ps:
                    if p.dtype != torch.float32:
                        raise TypeError("FusedAdamW: fp32 parameters only")
                    flat[o:o + p.numel()].copy_(p.detach().reshape(-1))
                    p.data = flat[o:o + p.numel()].view_as(p)
                    offs.append(o)
                    ns.append(p.numel())
                    o += p.numel()
            self._flat.append(dict(
                params=ps, flat=flat, grad=torch.zeros_like(flat), m=torch.zeros_like(flat),
                v=torch.zeros_like(flat), step=torch.zeros(1, dtype=torch.float32, device=dev),
                offs=(C.c_int64 * len(ps))(*offs), ns=(C.c_int64 * len(ps))(*ns)))

    def flat_params(self, group=0):
        return self._flat[group]["flat"]

    def flat_grad(self, group=0):
        return self._flat[group]["grad"]

    def pack_grads(self):
        """Gather every p.grad into the flat gradient buffer (one launch per 48 tensors)."""
        for fl in self._flat:
            if fl is None:
                continue
            ps = fl["params"]
            srcs = _lib.ptr_array([p.grad for p in ps])
            lib.pack(srcs, fl["offs"], fl["ns"], len(ps), fl["grad"].data_ptr(), 0, stream())

    def reduce_grads(self):
        """Run the gradient hook (the data-parallel all-reduce) on each flat gradient."""
        if self.grad_hook is not None:
            for fl in self._flat:
                if fl is not None:
                    self.grad_hook(fl["grad"])

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        self.pack_grads()
        self.reduce_grads()
        self.apply_update()
        return loss

    @torch.no_grad()
    def apply_update(self):
        """The AdamW update from the (already packed / reduced) flat gradient."""
        for group, fl in zip(self.param_groups, self._flat):
            if fl is None:
                continue
            b1, b2 = group["betas"]
            lib.step_advance(fl["step"].data_ptr(), None, stream())
            runs = self._runs(fl)
            for o, n in runs:
                lib.adamw(fl["flat"].data_ptr() + 4 * o, fl["grad"].data_ptr() + 4 * o,
                          fl["m"].data_ptr() + 4 * o, fl["v"].data_ptr() + 4 * o, n,
                          fl["step"].data_ptr(), float(group["lr"]), float(b1), float(b2),
                          float(group["eps"]), float(group["weight_decay"]), stream())

    @staticmethod
    def _runs(fl):
        runs, start, cur = [], None, 0
        for p, o, n in zip(fl["params"], fl["offs"], fl["ns"]):
            if p.grad is None:
                if start is not None:
                    runs.append((start, cur - start))
                    start = None
            elif start is None:
                start = o
            cur = o + n
        if start is not None:
            runs.append((start, cur - start))
        return runs
