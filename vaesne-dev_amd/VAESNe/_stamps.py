"""Device-side phase timestamps of the training step (VAESNE_STAMPS=1; tools/stamps.py).

A stamp is one single-thread node (vaesne_stamp) that writes the device's constant
100 MHz wall clock into a named slot when its stream reaches it: the phase
boundaries of a captured (replayed) step are timed with no tracer in the loop
(rocprofv3's per-dispatch cost stretches exactly the latency-bound encoder phases
one would want to see).  Off by default: with _config.stamps False, mark() launches
nothing and the captured graph is the product graph."""
import torch

from . import _config
from ._lib import lib, stream

NSLOT = 64
_slots = {}          # name -> slot (first use order)
_bufs = {}           # device index -> int64[NSLOT]


def mark(name):
    """Stamp `name` on the current stream (no-op unless VAESNE_STAMPS=1)."""
    if not _config.stamps or not torch.cuda.is_available():
        return
    dev = torch.cuda.current_device()
    buf = _bufs.get(dev)
    if buf is None:
        if torch.cuda.is_current_stream_capturing():
            return                     # never allocate inside a capture
        buf = _bufs[dev] = torch.zeros(NSLOT, dtype=torch.int64, device=f"cuda:{dev}")
    slot = _slots.get(name)
    if slot is None:
        if len(_slots) >= NSLOT:
            return
        slot = _slots[name] = len(_slots)
    lib.stamp(buf.data_ptr(), slot, stream())


def read(device=None):
    """{name: microseconds since the earliest stamp} of the last executed step."""
    dev = torch.cuda.current_device() if device is None else torch.device(device).index
    buf = _bufs.get(dev)
    if buf is None:
        return {}
    vals = buf.cpu().tolist()
    got = {n: vals[s] for n, s in _slots.items() if vals[s]}
    if not got:
        return {}
    t0 = min(got.values())
    return {n: (v - t0) / 100.0 for n, v in sorted(got.items(), key=lambda kv: kv[1])}
