"""Mixture-of-experts multimodal VAE over (light curve, spectrum) pairs,
MI355X build (reference: mmVAE.py:71-132, photospecMMVAE)."""
import contextlib

import torch
import torch.distributions as dist
import torch.nn as nn

from . import _config, _ops, _stamps
from .util_layers import ReferencePickle


_SIDE = {}


def _side_stream(t):
    """A second HIP stream for the photometry branch (_config.streams off: none)."""
    if not t.is_cuda or not _config.streams:
        return None
    dev = t.device.index if t.device.index is not None else torch.cuda.current_device()
    st = _SIDE.get(dev)
    if st is None:
        st = _SIDE[dev] = torch.cuda.Stream(device=dev)
    return st


def _tensors(obj):
    if isinstance(obj, torch.Tensor):
        return [obj]
    if isinstance(obj, (tuple, list)):
        return [t for o in obj for t in _tensors(o)]
    if hasattr(obj, "tensors"):
        return obj.tensors()
    return []


class _Branches:
    """Run branch 0 (photometry) on a side stream and branch 1 (spectra) on the
    current stream, then join.  The photometry encoder / decoder are chains of
    small latency-bound kernels; beside the spectra work they cost ~nothing.
    Host order (and so RNG call ids / injected noise order) is unchanged, and
    autograd replays each branch's backward on the stream its forward used."""

    def __init__(self, side):
        self.side = side
        self.main = torch.cuda.current_stream() if side is not None else None

    def __enter__(self):
        if self.side is not None:
            self.side.wait_stream(self.main)
        return self

    def on(self, branch):
        if self.side is None or branch != 0:
            return contextlib.nullcontext()
        return torch.cuda.stream(self.side)

    def to_side(self, *ts):
        """tensors made on the main stream that the side branch reads"""
        if self.side is not None:
            _ops.used_on(self.side, *ts)

    def to_main(self, *ts):
        """tensors the side branch made that the main stream reads"""
        if self.side is not None:
            _ops.used_on(self.main, *ts)

    def __exit__(self, *exc):
        if self.side is not None:
            self.main.wait_stream(self.side)
        return False


class _CellMatrix(list):
    """The 2x2 px_zs list of lists; `merged` holds the per-decoder (loc, scale)
    [K, 2B, L_d] tensors its cells are views of (empty if decoded per cell)."""

    def __init__(self, rows):
        super().__init__(rows)
        self.merged = []


class photospecMMVAE(ReferencePickle, nn.Module):
    def __init__(self, vaes, prior_dist=dist.Laplace, beta=1., length_ratio=982 / 60):
        super().__init__()
        self.pz = prior_dist
        self.vaes = nn.ModuleList(vaes)
        self.modelName = "photospectra"
        self._pz_params = nn.ParameterList([
            nn.Parameter(torch.zeros(vaes[0].latent_len, vaes[0].latent_dim), requires_grad=False),
            nn.Parameter(torch.ones(vaes[0].latent_len, vaes[0].latent_dim), requires_grad=False),
        ])
        # mmVAE.py:82-84
        self.vaes[0].llik_scaling = 1. / beta
        self.vaes[1].llik_scaling = 1. / beta
        self.vaes[0].llik_scaling *= length_ratio

    @property
    def pz_params(self):
        return self._pz_params

    def forward(self, x, K=1):
        """mmVAE.py:91-106: px_zs[e][d] = vaes[d].decode(zs_e, x[d]) for every
        (encoder e, decoder d) pair; the diagonal is each VAE's own forward.

        The posteriors are drawn in the reference's order (photometry first,
        so injected / seeded noise lines up).  Then each decoder runs ONCE over
        both modalities' latents, batch-concatenated ([K, 2B]): per-sample the
        arithmetic is the reference's, and the step launches every decoder
        kernel once instead of twice (and needs no gradient sums over two
        decoder calls).  px_zs cells are views of those [K, 2B, L] tensors;
        `px_zs.merged` lets the fused m_iwae read them in place."""
        n = len(self.vaes)
        side = _side_stream(x[0][0]) if n == 2 else None
        merged = all((v.latent_len, v.latent_dim) == (self.vaes[0].latent_len,
                                                       self.vaes[0].latent_dim) for v in self.vaes)
        # The decoders' input embeddings, first in-projections and block-1 self-attention
        # read only the decoder input grids (util_layers.decoder_stack_first), not the
        # latents: they are issued on the photometry stream BEFORE the photometry encoder,
        # so they run beside the latency-bound spectra encoder (A/B 9.96 -> 9.61 ms per
        # step), and autograd (which runs the later-created of two ready nodes first)
        # issues the photometry encoder's backward ahead of the block-1 attention
        # backwards on that stream (A/B 9.51 -> 9.43 ms).  Without a side stream they
        # run first on the current stream.
        preps = [None] * n
        prep_ok = merged and all(hasattr(v, "decode_prepare") for v in self.vaes)
        qz_xs, zss = [None] * n, [None] * n
        _stamps.mark("fwd")
        with _Branches(side) as br:
            br.to_side(*x[0])
            for m, vae in enumerate(self.vaes):
                with br.on(m):
                    if m == 0 and prep_ok:
                        br.to_side(*x[1])
                        for d in range(n):
                            preps[d] = self.vaes[d].decode_prepare(x[d], K, groups=n)
                        _stamps.mark("side:dec_prepare")
                    qz_xs[m], zss[m] = vae.posterior(x[m], K=K)
                    _stamps.mark(f"enc{m}")
            br.to_main(qz_xs[0].loc, qz_xs[0].scale, zss[0], *_tensors(preps))
        _stamps.mark("encoders_joined")
        px_zs = _CellMatrix([[None for _ in range(n)] for _ in range(n)])
        if all(z.shape == zss[0].shape for z in zss):
            B = zss[0].shape[1]
            # one zcat alias per decoder and the zs for the loss: their gradients meet in
            # one kernel (_ops.latent_cat) instead of autograd's adds
            zcats, zss = _ops.latent_cat(zss, n)
            zss = list(zss)
            px_zs.merged = [None] * n
            with _Branches(side) as br:
                br.to_side(*zcats, *_tensors(preps))
                for d in range(n):
                    vae = self.vaes[d]
                    with br.on(d):
                        px_zs.merged[d] = vae.decode_params(zcats[d], x[d], groups=n,
                                                            prepared=preps[d])
                        _stamps.mark(f"dec{d}")
                br.to_main(*px_zs.merged[0])
            _stamps.mark("decoders_joined")
            for d, vae in enumerate(self.vaes):
                loc, scale = px_zs.merged[d]
                for e in range(n):
                    px_zs[e][d] = vae._dist(vae.px_z, loc[:, e * B:(e + 1) * B],
                                            scale[:, e * B:(e + 1) * B])
        else:   # latent shapes differ per modality: one decoder call per cell
            for e, zs in enumerate(zss):
                for d, vae in enumerate(self.vaes):
                    px_zs[e][d] = vae.decode(zs, x[d])
        return qz_xs, px_zs, zss

    def generate(self, N, x):
        """mmVAE.py:108-118: N prior draws per conditioning example, decoded by
        every modality."""
        self.eval()
        with torch.no_grad():
            B = x[0][0].shape[0]
            loc = self._pz_params[0].expand(B, *self._pz_params[0].shape).contiguous()
            scale = self._pz_params[1].expand(B, *self._pz_params[1].shape).contiguous()
            latents = _ops.laplace_rsample(loc, scale, N)
            return [vae.decode(latents, x[d]).mean for d, vae in enumerate(self.vaes)]

    def reconstruct(self, data, K=1):
        """mmVAE.py:120-126: cross-modal matrix of reconstruction means."""
        self.eval()
        with torch.no_grad():
            _, px_zs, _ = self.forward(data, K=K)
            return [[px_z.mean for px_z in r] for r in px_zs]
