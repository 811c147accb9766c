"""FusedAdamW: torch.optim.AdamW arithmetic (the cannon scripts' optimizer,
e.g. cannon/test_photospectra.py:133, cannon/ZTF_photospect.py:119) over one
flat fp32 parameter buffer on the device.

* Parameters are re-bound as views into one flat buffer (module identity and
  state_dict keys unchanged), so the update is ONE HIP kernel launch and the
  gradient is ONE flat buffer — the unit the data-parallel all-reduce moves.
* The step counters live on the device, so a whole training step (forward,
  backward, pack, all-reduce, update) can be captured in one hipGraph.
* As in torch.optim.AdamW, every parameter has its own step count, advanced only
  when it has a gradient, and parameters whose .grad is None are skipped.
* state_dict() / load_state_dict() use torch.optim.AdamW's format (per-parameter
  "step", "exp_avg", "exp_avg_sq"), so checkpoints move between the two.  Only
  lr / betas / eps / weight_decay are taken from a loaded group; a group saved with
  amsgrad or maximize set is refused (the kernel implements neither).
* Non-finite guard: inside training_step the update kernels read the device flag of
  VAESNe.guard (apply_update's `skip`) and apply nothing (parameters, moments and
  step counts unchanged) once a batch's forward flagged a NaN posterior or a
  non-finite loss; training_step raises on it.  A plain `step()` (a custom loop, as
  the reference's *2goldstein_* scripts write) updates unconditionally, exactly as
  torch.optim.AdamW would: a flag left by an earlier eval forward never silently
  drops its updates.
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
            pidx = torch.repeat_interleave(torch.arange(len(ps), dtype=torch.int32),
                                           torch.tensor(ns, dtype=torch.int64)).to(dev)
            # the gradient buffer carries 4 spare words: training_step's data-parallel
            # exchange all-reduces [gradient | loss | guard words] in place (distributed.FlatExchange)
            gstore = torch.zeros(n + 4, dtype=torch.float32, device=dev)
            self._flat.append(dict(
                params=ps, flat=flat, grad=gstore[:n], gstore=gstore, m=torch.zeros_like(flat),
                v=torch.zeros_like(flat),
                steps=torch.zeros(len(ps), dtype=torch.float32, device=dev), pidx=pidx,
                active={}, offs=(C.c_int64 * len(ps))(*offs), ns=(C.c_int64 * len(ps))(*ns)))

    def flat_params(self, group=0):
        return self._flat[group]["flat"]

    def flat_grad(self, group=0):
        return self._flat[group]["grad"]

    def flat_params_list(self):
        """Every parameter of the flat buffers, group after group, in buffer order (the
        layout of training_step's data-parallel gradient buffer)."""
        return [p for fl in self._flat if fl is not None for p in fl["params"]]

    def exchange_buffer(self):
        """The one group's gradient storage with its spare words (None with several groups)."""
        fls = [fl for fl in self._flat if fl is not None]
        return fls[0]["gstore"] if len(fls) == 1 else None

    def flat_sizes(self):
        """Elements per group's flat buffer (0 for a group without trainable tensors)."""
        return [0 if fl is None else fl["flat"].numel() for fl in self._flat]

    def pack_grads(self):
        """Gather every p.grad into the flat gradient buffer (one launch per 144 tensors)."""
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
    def apply_update(self, skip=None, grads=None):
        """The AdamW update from the (already packed / reduced) flat gradient.
        skip: device address of two int32 words (the guard flag, or the all-reduced
        guard words of training_step's data-parallel exchange); when either is set the
        kernels change nothing.  Only training_step passes it: a plain step() updates
        unconditionally, as torch.optim.AdamW does.  grads: per group, a flat gradient
        to read instead of the packed one (training_step's all-reduced buffer)."""
        for gi, (group, fl) in enumerate(zip(self.param_groups, self._flat)):
            if fl is None:
                continue
            b1, b2 = group["betas"]
            gflat = fl["grad"] if grads is None else grads[gi]
            if gflat.numel() != fl["flat"].numel() or not gflat.is_contiguous():
                raise ValueError("FusedAdamW.apply_update: flat gradient of the wrong size")
            lib.adamw_steps_advance(fl["steps"].data_ptr(), self._active(fl), len(fl["params"]),
                                    skip, stream())
            runs = self._runs(fl)
            for o, n in runs:
                lib.adamw(fl["flat"].data_ptr() + 4 * o, gflat.data_ptr() + 4 * o,
                          fl["m"].data_ptr() + 4 * o, fl["v"].data_ptr() + 4 * o, n,
                          fl["steps"].data_ptr(), fl["pidx"].data_ptr() + 4 * o,
                          float(group["lr"]), float(b1), float(b2),
                          float(group["eps"]), float(group["weight_decay"]), skip, stream())

    @staticmethod
    def _active(fl):
        """Device mask of the parameters with a gradient (None: all), cached per pattern;
        built from pinned memory so a graph capture can record the copy."""
        flags = tuple(p.grad is not None for p in fl["params"])
        if all(flags):
            return None
        t = fl["active"].get(flags)
        if t is None:
            host = torch.tensor(flags, dtype=torch.uint8).pin_memory()
            t = (host, host.to(fl["steps"].device, non_blocking=True))
            fl["active"][flags] = t
        return t[1].data_ptr()

    # ---- torch.optim.AdamW-format state --------------------------------------
    def state_dict(self):
        state, groups, base = {}, [], 0
        for group, fl in zip(self.param_groups, self._flat):
            g = {k: v for k, v in group.items() if k != "params"}
            g["params"] = list(range(base, base + len(group["params"])))
            groups.append(g)
            if fl is not None:
                steps = fl["steps"].cpu()
                index = {id(p): i for i, p in enumerate(group["params"])}
                for j, (p, o, n) in enumerate(zip(fl["params"], fl["offs"], fl["ns"])):
                    if float(steps[j]) == 0.0:
                        continue        # never updated: no state, as in torch
                    state[base + index[id(p)]] = {
                        "step": steps[j].clone(),
                        "exp_avg": fl["m"][o:o + n].view_as(p).clone(),
                        "exp_avg_sq": fl["v"][o:o + n].view_as(p).clone()}
            base += len(group["params"])
        return {"state": state, "param_groups": groups}

    def load_state_dict(self, state_dict):
        groups = state_dict["param_groups"]
        if len(groups) != len(self.param_groups):
            raise ValueError("loaded state dict has a different number of parameter groups")
        st = state_dict["state"]
        for group, saved, fl in zip(self.param_groups, groups, self._flat):
            if len(saved["params"]) != len(group["params"]):
                raise ValueError("loaded state dict contains a parameter group that doesn't "
                                 "match the size of optimizer's group")
            for k in ("amsgrad", "maximize"):
                if saved.get(k, False):
                    raise ValueError(f"FusedAdamW: the loaded optimizer state has {k}=True, "
                                     "which the fused AdamW kernel does not implement")
            for k in ("lr", "betas", "eps", "weight_decay"):
                if k in saved:
                    group[k] = tuple(saved[k]) if k == "betas" else saved[k]
            if fl is None:
                continue
            where = {id(p): j for j, p in enumerate(fl["params"])}
            steps = torch.zeros(len(fl["params"]), dtype=torch.float32)
            with torch.no_grad():
                for p, key in zip(group["params"], saved["params"]):
                    j = where.get(id(p))
                    if j is None:
                        continue
                    o, n = fl["offs"][j], fl["ns"][j]
                    s = st.get(key, st.get(str(key)))
                    if s is None:
                        fl["m"][o:o + n].zero_()
                        fl["v"][o:o + n].zero_()
                        continue
                    steps[j] = float(s["step"])
                    fl["m"][o:o + n].copy_(s["exp_avg"].reshape(-1))
                    fl["v"][o:o + n].copy_(s["exp_avg_sq"].reshape(-1))
            fl["steps"].copy_(steps)

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
