"""Non-finite detection for the VAESNe step without an extra host sync.

The reference stops when a posterior parameter is NaN (PhotometricVAE.py:160-161,
ImageVAE.py:193-194: `torch.isnan(...).any()` then `breakpoint()`), which on a GPU
is a device->host sync inside every forward, and BEFORE the optimizer update.
Here the kernels that produce the posterior parameters (latent head) and the
losses (m_iwae's log-mean-exp sum, elbo) set a device flag `int32[2]` instead:

    flag[0] = 1   some posterior loc / scale was NaN (the reference's test)
    flag[1] = 1   the loss was NaN or Inf (stricter than the reference, which
                  would carry on with a non-finite loss)

Who reads it:
  * the FusedAdamW kernels (vaesne_adamw / vaesne_adamw_steps_advance `skip`):
    a flagged step changes neither the parameters nor the step counts, also
    inside a captured hipGraph;
  * `training_step`: resets the flag before each batch's forward, reads it at one
    sync placed BEFORE `optimizer.step()` (folded into the data-parallel loss
    all-reduce, so every rank raises together: a rank-local raise would leave the
    others blocked in the next all-reduce), and raises RuntimeError (never pdb);
  * `check()` for other callers.
"""
from __future__ import annotations

import torch

_flags: dict = {}

_WHAT = {0: "posterior location / scale (encoder output, NaN)", 1: "loss (NaN / Inf)"}


def flag(device) -> torch.Tensor:
    """The device int32[2] flag of `device` (created zeroed on first use)."""
    device = torch.device(device)
    key = device.index if device.index is not None else torch.cuda.current_device()
    f = _flags.get(key)
    if f is None:
        f = _flags[key] = torch.zeros(2, dtype=torch.int32, device=torch.device("cuda", key))
    return f


def ptr(t: torch.Tensor):
    """Flag pointer for the device tensor t lives on (None for host tensors)."""
    return flag(t.device).data_ptr() if t.is_cuda else None


def status(device) -> tuple:
    """(posterior_nonfinite, loss_nonfinite) — synchronises with the device."""
    f = flag(device).tolist()
    return bool(f[0]), bool(f[1])


def reset(device):
    device = torch.device(device)
    if device.type == "cuda":
        flag(device).zero_()


def words(device) -> torch.Tensor:
    """The flag as float32[2] on `device` (zeros for host devices), for folding into
    a loss all-reduce; no sync."""
    device = torch.device(device)
    if device.type != "cuda":
        return torch.zeros(2, dtype=torch.float32, device=device)
    return flag(device).float()


def raise_for(device, bad, where: str = "VAESNe"):
    """Raise RuntimeError for the (posterior, loss) flags `bad` (clearing the device
    flag first, so training can be resumed after handling)."""
    if any(bad):
        reset(device)
        what = " and ".join(_WHAT[i] for i, b in enumerate(bad) if b)
        raise RuntimeError(f"{where}: non-finite {what}; the reference stops here "
                           "(PhotometricVAE.py:160-161); the update was not applied")


def check(device, where: str = "VAESNe"):
    """Raise RuntimeError if a kernel flagged a non-finite value since the last
    check (the flag is cleared first)."""
    device = torch.device(device)
    if device.type != "cuda":
        return
    key = device.index if device.index is not None else torch.cuda.current_device()
    if key not in _flags:
        return
    raise_for(device, status(device), where)
