"""Non-finite detection for the VAESNe step without an extra host sync.

The reference stops when a posterior parameter is NaN (PhotometricVAE.py:160-161,
ImageVAE.py:193-194: `torch.isnan(...).any()` then `breakpoint()`), which on a GPU
is a device->host sync inside every forward.  Here the kernels that produce the
posterior parameters (latent head) and the losses (m_iwae's log-mean-exp sum,
elbo) set a device flag `int32[2]` instead:

    flag[0] = 1   some posterior loc / scale was NaN or Inf
    flag[1] = 1   the loss was NaN or Inf

`training_step` reads it right after the `.item()` it already does
(training_util.py:46 in the reference), when the stream is drained anyway, and
raises RuntimeError (never pdb).  `check()` does the same for other callers.
"""
from __future__ import annotations

import torch

_flags: dict = {}

_WHAT = {0: "posterior location / scale (encoder output)", 1: "loss"}


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
    flag(device).zero_()


def check(device, where: str = "VAESNe"):
    """Raise RuntimeError if a kernel flagged a non-finite value since the last
    check (the flag is cleared first, so training can be resumed after handling)."""
    device = torch.device(device)
    if device.type != "cuda":
        return
    key = device.index if device.index is not None else torch.cuda.current_device()
    if key not in _flags:
        return
    bad = status(device)
    if any(bad):
        reset(device)
        what = " and ".join(_WHAT[i] for i, b in enumerate(bad) if b)
        raise RuntimeError(f"{where}: non-finite {what} (NaN / Inf); the reference stops here "
                           "(PhotometricVAE.py:160-161)")
