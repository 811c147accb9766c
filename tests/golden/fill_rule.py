"""Deterministic parameter fill and synthetic inputs shared by the golden
generator (run against the reference) and by the tests (run against the oracle
and the HIP build).  Pure numpy: importable from either side without touching
a package called ``VAESNe``.

Fill rule (by state_dict key, so module construction order does not matter):
  rng = default_rng(crc32(key))
  * '_pz_params.*'              -> None (keep the reference's zeros/ones)
  * LayerNorm weight            -> 1 + 0.1 N(0,1)
  * LayerNorm / Linear bias     -> 0.1 N(0,1)
  * >= 2-D weights              -> N(0,1) / sqrt(fan_in)   (fan_in = prod(shape[1:]):
                                   Linear in_features, Conv2d in_channels * kh * kw)
  * initbottleneck              -> N(0,1)
Inputs follow SURVEY.md §8(d).
"""
import zlib

import numpy as np


def fill(key: str, shape):
    if "_pz_params" in key:
        return None
    rng = np.random.default_rng(zlib.crc32(key.encode()))
    z = rng.standard_normal(shape)
    last = key.split(".")[-1]
    if ("layernorm" in key) and last == "weight":
        v = 1.0 + 0.1 * z
    elif last.endswith("bias"):
        v = 0.1 * z
    elif key.endswith("initbottleneck"):
        v = z
    elif len(shape) >= 2:
        v = z / np.sqrt(np.prod(shape[1:]))
    else:
        v = z
    return v.astype(np.float32)


def photo_inputs(rng, B, L, nb, p_mask=0.1):
    """LC flux ~ N(0,1); time sorted N(0,1) per row; band ~ U{0..nb-1};
    mask ~ Bernoulli(p) (True = unobserved) with >= 1 observed per row."""
    flux = rng.standard_normal((B, L)).astype(np.float32)
    time = np.sort(rng.standard_normal((B, L)), axis=1).astype(np.float32)
    band = rng.integers(0, nb, size=(B, L)).astype(np.int64)
    mask = rng.random((B, L)) < p_mask
    mask[:, 0] = False
    return flux, time, band, mask


def spec_inputs(rng, B, L, p_mask=0.05):
    """spectrum flux ~ N(0,1); wavelength = linspace(-1.7, 1.7, L) per row;
    phase ~ N(0,1); mask ~ Bernoulli(p) with >= 1 observed per row."""
    flux = rng.standard_normal((B, L)).astype(np.float32)
    wavelength = np.tile(np.linspace(-1.7, 1.7, L, dtype=np.float32), (B, 1))
    phase = rng.standard_normal((B,)).astype(np.float32)
    mask = rng.random((B, L)) < p_mask
    mask[:, 0] = False
    return flux, wavelength, phase, mask


def image_inputs(rng, B, C, H):
    """images ~ U(0, 1) [B, C, H, H] (MNIST-like intensities, cannon/mnist.py:13-16
    ToTensor range) and the loader's label column (unused by the model)."""
    img = rng.random((B, C, H, H)).astype(np.float32)
    label = np.zeros((B,), dtype=np.int64)
    return img, label
