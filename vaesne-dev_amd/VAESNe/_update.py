"""The optimizer update of `training_step`, enqueued behind a device-side skip.

The reference reads each batch's loss with `.item()` right after `optimizer.step()`
(training_util.py:44-46) and stops in pdb on a NaN posterior inside the forward
(PhotometricVAE.py:160-161), i.e. a flagged batch never reaches the parameters.
Reading the verdict before every update (as round 3 did) leaves the GPU idle while
the host launches the update and the next batch.  Here the update is enqueued at once
and guarded on the device instead:

  * the non-finite flag of VAESNe.guard is STICKY for the whole training_step call
    (cleared once at its start): from the first flagged batch on, every update kernel
    of the call is a no-op;
  * the host reads each batch's (loss, flags) two batches late, while the next two
    run, and raises there; the host-side bookkeeping of the updates that the device
    skipped (torch.optim.AdamW's per-parameter `state['step']`) is rolled back, so
    the optimizer is exactly as it was before the flagged batch.

Updaters (chosen once per optimizer):
  FusedUpdater       VAESNe.optim.FusedAdamW: its flat kernels with `skip`.
  TorchAdamWUpdater  the scripts' own `torch.optim.AdamW(params, lr)`
                     (cannon/ZTF_photospect.py:119): torch's foreach update applied op
                     for op by `vaesne_adamw_list` on the optimizer's own state tensors,
                     with the scalars torch computes on the host, so `state_dict()`,
                     checkpoints and later plain `step()` calls are torch's own.
                     Only for the configuration torch runs that way (float32 dense
                     tensors, no amsgrad / maximize / capturable / differentiable /
                     fused, no step hooks, `step` not patched).
  Updater            anything else: the optimizer's own `step()` after the host has
                     read the batch's verdict (the round-3 behaviour).
"""
from __future__ import annotations

import collections
import ctypes as C

import torch

from . import _lib
from .optim import FusedAdamW

# vaesne_adamw_list `fma`: torch's foreach kernels as ROCm's compiler builds them
# contract a + b*c into one fused multiply-add (tests/test_gpu_optim.py checks the
# kernel bitwise against torch.optim.AdamW)
TORCH_FMA = 1


class Updater:
    """The optimizer's own step(), after the verdict (no device-side skip)."""

    device_skip = False

    def __init__(self, optimizer):
        self.opt = optimizer

    def layout(self):
        """The parameters in the order of the data-parallel gradient buffer."""
        return [p for g in self.opt.param_groups for p in g["params"] if p.requires_grad]

    def ready(self) -> bool:
        """Whether this batch's update can be enqueued behind the device skip."""
        return False

    def update(self, skip=None, flat=None):
        self.opt.step()

    def rollback(self, n):
        pass


class FusedUpdater(Updater):
    device_skip = True

    def layout(self):
        return self.opt.flat_params_list()

    def ready(self):
        return True

    def update(self, skip=None, flat=None):
        grads = None
        if flat is None:
            self.opt.pack_grads()
        else:           # the all-reduced buffer, group after group
            grads, o = [], 0
            for n in self.opt.flat_sizes():
                grads.append(flat[o:o + n])
                o += n
        self.opt.apply_update(skip=skip, grads=grads)


def _hooks_free(opt):
    from torch.optim import optimizer as O
    return not (getattr(opt, "_optimizer_step_pre_hooks", None)
                or getattr(opt, "_optimizer_step_post_hooks", None)
                or getattr(O, "_global_optimizer_pre_hooks", None)
                or getattr(O, "_global_optimizer_post_hooks", None))


class TorchAdamWUpdater(Updater):
    device_skip = True

    @staticmethod
    def supports(opt) -> bool:
        if type(opt) is not torch.optim.AdamW or "step" in opt.__dict__ or not _hooks_free(opt):
            return False
        for g in opt.param_groups:
            if g.get("amsgrad") or g.get("maximize") or g.get("capturable") \
                    or g.get("differentiable") or g.get("fused") or g.get("foreach") is False:
                return False
            if g.get("decoupled_weight_decay", True) is False:
                return False
            if any(torch.is_tensor(g[k]) for k in ("lr", "weight_decay", "eps")) \
                    or any(torch.is_tensor(b) for b in g["betas"]):
                return False
        return True

    def __init__(self, optimizer):
        super().__init__(optimizer)
        self.hist = collections.deque(maxlen=8)
        self._bkey = None      # identity key of the last validated batch (_batch)
        self._bval = None
        self._arrays = None    # (identity key, ctypes arrays) of the last launch (update)
        self._fast = None      # steady-state plan of the cached batch (_fast_plan)
        self._arrays_bkey = None   # the batch key the launch arrays were last checked for

    def _batch(self):
        """(params, grads, states) of the tensors torch would update now, or None if
        one of them is outside the supported configuration.  A batch of the same tensors
        as the previous one (the captured step's gradients, the same state tensors) is
        not re-validated."""
        st_of = self.opt.state
        key = []
        for group in self.opt.param_groups:
            for p in group["params"]:
                g = p.grad
                if g is not None:
                    st = st_of.get(p)
                    key.append((id(p), id(g), id(st["exp_avg"]) if st else 0, p.data_ptr(),
                                g.data_ptr()))
        key = tuple(key)
        if key == self._bkey:
            return list(self._bval)
        out = self._batch_full()
        self._bkey, self._bval = (key, tuple(out)) if out is not None else (None, None)
        return out

    def _batch_full(self):
        out = []
        for gi, group in enumerate(self.opt.param_groups):
            for p in group["params"]:
                g = p.grad
                if g is None:
                    continue
                if not (p.is_cuda and p.dtype == torch.float32 and g.dtype == torch.float32
                        and not g.is_sparse and p.is_contiguous() and g.is_contiguous()
                        and g.device == p.device and p.numel() < 2 ** 31):
                    return None
                st = self.opt.state.get(p)
                if st and not (st["exp_avg"].is_contiguous() and st["exp_avg_sq"].is_contiguous()
                               and not st["step"].is_cuda):
                    return None
                out.append((gi, p, g))
        return out

    def ready(self):
        # a scheduler that patches step() or a hook registered since: torch's own step()
        if "step" in self.opt.__dict__ or not _hooks_free(self.opt):
            self._pending = None
        else:
            self._pending = self._batch()
        return self._pending is not None

    def _fast_plan(self, batch):
        """Steady state (the cached batch again, every state created, one step count per
        parameter group, the cached launch arrays built for it): the per-parameter step
        tensors become views of ONE host tensor, so a batch's host bookkeeping is one add and
        one read instead of a loop over the parameters.  None when not in that state."""
        f = self._fast
        st_of = self.opt.state
        if f is not None and f["key"] == self._bkey and f["akey"] == self._arrays[0]:
            if all(st_of[p]["step"] is t for (_, p, _), t in zip(batch, f["steps"])):
                return f
        sts = [st_of.get(p) for _, p, _ in batch]
        # the cached launch arrays must be this batch's (built by the general path for it)
        if self._bkey is None or self._arrays_bkey != self._bkey or any(not st for st in sts):
            return None
        gis = [gi for gi, _, _ in batch]
        vals = [float(st["step"]) for st in sts]
        per_group = {}
        for gi, v in zip(gis, vals):
            if per_group.setdefault(gi, v) != v:
                return None
        order = list(per_group)                         # first appearance: the general path's
        if tuple(order.index(gi) for gi in gis) != self._arrays[0][5]:   # set numbering
            return None
        base = torch.tensor(vals, dtype=torch.float32)
        steps = []
        for k, st in enumerate(sts):
            st["step"] = base[k]          # a view: torch's own step() updates it in place too
            steps.append(st["step"])
        self._fast = {"key": self._bkey, "akey": self._arrays[0], "base": base, "steps": steps,
                      "order": order, "first": [gis.index(gi) for gi in order],
                      "stepped": [(p, False) for _, p, _ in batch]}
        return self._fast

    def _fast_update(self, f, skip):
        base = f["base"]
        base.add_(1.0)
        try:
            vals = base.tolist()
            groups = self.opt.param_groups
            coefs = []
            for gi, k in zip(f["order"], f["first"]):
                step = vals[k]
                grp = groups[gi]
                lr, wd, eps = grp["lr"], grp["weight_decay"], grp["eps"]
                b1, b2 = grp["betas"]
                bc1 = 1 - b1 ** step
                bc2 = 1 - b2 ** step
                coefs += [1 - lr * wd, 1 - b1, b2, 1 - b2, bc2 ** 0.5, eps, (lr / bc1) * -1, 0.0]
            pa, ga, ma, va, na, sa = self._arrays[1]
            _lib.lib.adamw_list(pa, ga, ma, va, na, sa, (C.c_float * len(coefs))(*coefs),
                                len(f["steps"]), skip, TORCH_FMA, _lib.stream())
        except BaseException:
            base.sub_(1.0)                # the step counts never run ahead of launched updates
            raise
        self.hist.append(f["stepped"])

    def update(self, skip=None, flat=None):
        batch = self._pending
        self._pending = None
        if not batch:
            self.hist.append([])
            return
        f = self._fast_plan(batch) if self._arrays is not None else None
        if f is not None:
            self._fast_update(f, skip)
            return
        groups = self.opt.param_groups
        ps, gs, ms, vs, ns, sets = [], [], [], [], [], []
        coefs, set_of, stepped, steps = [], {}, [], []
        added = False
        try:
            for gi, p, g in batch:
                st = self.opt.state[p]
                created = len(st) == 0
                if created:       # torch's lazy state (torch/optim/adam.py _init_group)
                    st["step"] = torch.tensor(0.0, dtype=torch.float32)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                steps.append(st["step"])
                stepped.append((p, created))
            # every step count += 1 and read back in three host ops, not two per parameter (the
            # per-tensor add and item() were most of the loop's host time at small batches)
            torch._foreach_add_(steps, 1.0)
            added = True
            step_vals = torch.stack(steps).tolist()
            for (gi, p, g), step in zip(batch, step_vals):
                st = self.opt.state[p]
                key = (gi, step)
                k = set_of.get(key)
                if k is None:
                    grp = groups[gi]
                    lr, wd, eps = grp["lr"], grp["weight_decay"], grp["eps"]
                    b1, b2 = grp["betas"]
                    bc1 = 1 - b1 ** step
                    bc2 = 1 - b2 ** step
                    k = set_of[key] = len(set_of)
                    coefs += [1 - lr * wd, 1 - b1, b2, 1 - b2, bc2 ** 0.5, eps, (lr / bc1) * -1, 0.0]
                ps.append(p)
                gs.append(g)
                ms.append(st["exp_avg"])
                vs.append(st["exp_avg_sq"])
                ns.append(p.numel())
                sets.append(k)
            n = len(ps)
            # the arrays hold device addresses: keyed by the addresses themselves
            akey = (tuple(t.data_ptr() for t in ps), tuple(t.data_ptr() for t in gs),
                    tuple(t.data_ptr() for t in ms), tuple(t.data_ptr() for t in vs), tuple(ns),
                    tuple(sets))
            if self._arrays is None or self._arrays[0] != akey:
                self._arrays = (akey, (_lib.ptr_array(ps), _lib.ptr_array(gs), _lib.ptr_array(ms),
                                       _lib.ptr_array(vs), (C.c_int64 * n)(*ns), (C.c_int32 * n)(*sets)))
            self._arrays_bkey = self._bkey
            pa, ga, ma, va, na, sa = self._arrays[1]
            _lib.lib.adamw_list(pa, ga, ma, va, na, sa, (C.c_float * len(coefs))(*coefs), n,
                                skip, TORCH_FMA, _lib.stream())
        except BaseException:
            # anything failing between the lazy state creation and a completed enqueue (a
            # stack of step tensors on different devices, a missing group key, a checked
            # hipError partway): undo this update's host bookkeeping, so the step counts
            # never run ahead of launched updates
            for p, created in stepped:
                st = self.opt.state[p]
                if added:
                    st["step"] -= 1
                if created:
                    del self.opt.state[p]
            raise
        self.hist.append(stepped)

    def rollback(self, n):
        """Undo the host bookkeeping of the last n updates (the device skipped them)."""
        for _ in range(min(n, len(self.hist))):
            for p, created in self.hist.pop():
                st = self.opt.state[p]
                st["step"] -= 1
                if created:
                    del self.opt.state[p]


def for_optimizer(optimizer) -> Updater:
    """The updater of `optimizer` (cached on it)."""
    u = getattr(optimizer, "_vaesne_updater", None)
    if u is None or u.opt is not optimizer:
        if isinstance(optimizer, FusedAdamW):
            u = FusedUpdater(optimizer)
        elif TorchAdamWUpdater.supports(optimizer):
            u = TorchAdamWUpdater(optimizer)
        else:
            u = Updater(optimizer)
        optimizer._vaesne_updater = u
    return u
