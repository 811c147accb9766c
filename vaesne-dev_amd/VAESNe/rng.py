"""Random numbers of the VAESNe step.

Two consumers draw randomness in the reference: Laplace.rsample's uniform
draw (torch/distributions/laplace.py:83, one per VAE forward, photometry
first) and dropout (nn.Dropout / MHA attention dropout, util_layers.py:263-284).

Here every draw is counter-based on the device: a device int64[2]
{seed, counter} plus a host-side call id per call site.  The forward and
backward of one op share a call id, so dropout masks are regenerated, never
stored.  `advance()` bumps the device counter (used once per captured
training step so a replayed hipGraph draws fresh numbers).

Parity with the reference's RNG stream (identical seeds) is available for the
sampler: `inject_uniform([u_photo, u_spec])` makes the next rsample calls
consume the given draws in order, and `set_mode("torch_cpu")` draws u with
torch's CPU generator exactly as the reference does on CPU.  Dropout masks
cannot match torch's bernoulli stream bitwise; parity is defined with dropout
off.
"""
from __future__ import annotations

import contextlib

import torch

from . import _lib

_states: dict = {}
_seed = None
_call = 0
_drawn = False      # a call id was issued since the device counter last advanced
_queue: list = []
_mode = "device"


_MASK63 = (1 << 63) - 1


def rank_seed(seed: int, rank: int) -> int:
    """The device seed of data-parallel rank `rank` for a user seed: rank 0 keeps
    it, other ranks fold their rank in (a 64-bit Weyl step), so ranks that all
    called torch.manual_seed(0) — as every cannon script does, e.g.
    ZTF_photospect.py:19 — still draw their own Laplace noise and dropout masks
    (SURVEY.md §8(e)), while a single process is unchanged."""
    return (int(seed) ^ ((int(rank) * 0x9E3779B97F4A7C15) & _MASK63)) & _MASK63


def _rank() -> int:
    from . import distributed as D
    return D.env_world()[0]


def _default_seed() -> int:
    return rank_seed(int(torch.initial_seed()) & _MASK63, _rank())


def effective_seed() -> int:
    """The seed the device streams use (created on first use)."""
    global _seed
    if _seed is None:
        _seed = _default_seed()
    return _seed


def manual_seed(seed: int):
    """Reset the device RNG of every device to `seed` (folded with the
    data-parallel rank, see rank_seed), counter 0."""
    global _seed, _call, _drawn
    _seed = rank_seed(int(seed) & _MASK63, _rank())
    _call = 0
    _drawn = False
    for st in _states.values():
        st.copy_(torch.tensor([_seed, 0], dtype=torch.int64))


def state(device) -> torch.Tensor:
    """The device int64[2] {seed, counter} tensor (created lazily)."""
    global _seed
    device = torch.device(device)
    key = device.index if device.index is not None else torch.cuda.current_device()
    st = _states.get(key)
    if st is None:
        st = torch.tensor([effective_seed(), 0], dtype=torch.int64, device=torch.device("cuda", key))
        _states[key] = st
    return st


def next_call_id() -> int:
    global _call, _drawn
    _call = (_call + 1) & 0xFFFFFFFF
    _drawn = True
    return _call


def reset_call_ids():
    """Restart call ids (done at the top of a captured step so replays reuse them)."""
    global _call
    _call = 0


def advance(device, step: torch.Tensor | None = None):
    """Bump the device counter (and an optional device step counter)."""
    global _drawn
    st = state(device)
    _lib.lib.step_advance(_lib.ptr(step), st.data_ptr(), _lib.stream())
    _drawn = False


def begin_training(device):
    """training_step restarts the call ids at every batch; draws made since the last
    counter advance (an eval / generate / reconstruct call) used the current counter
    with call ids 1.., which the first training batch would repeat: advance past them."""
    if _drawn:
        advance(device)


def capturable() -> bool:
    """Whether the next draws may be captured in a hipGraph (device counter-based:
    no injected draws queued, not the host generator mode)."""
    return _mode == "device" and not _queue


def set_mode(mode: str):
    global _mode
    if mode not in ("device", "torch_cpu"):
        raise ValueError(mode)
    _mode = mode


@contextlib.contextmanager
def inject_uniform(us):
    """Within the block, rsample consumes these uniform draws (in order)."""
    n0 = len(_queue)
    _queue.extend(us)
    try:
        yield
    finally:
        del _queue[n0:]


def draw_uniform(shape, device) -> torch.Tensor:
    """u ~ U(eps-1, 1) of the given shape on `device` (laplace.py:83)."""
    shape = tuple(int(s) for s in shape)
    if _queue:
        u = _queue.pop(0)
        if tuple(u.shape) != shape:
            raise RuntimeError(f"injected uniform has shape {tuple(u.shape)}, need {shape}")
        return u.to(device=device, dtype=torch.float32).contiguous()
    if _mode == "torch_cpu":
        eps = torch.finfo(torch.float32).eps
        return torch.empty(shape).uniform_(eps - 1, 1).to(device)
    u = torch.empty(shape, device=device, dtype=torch.float32)
    n = u.numel()
    _lib.lib.uniform(u.data_ptr(), n, state(device).data_ptr(), next_call_id(), _lib.stream())
    return u
