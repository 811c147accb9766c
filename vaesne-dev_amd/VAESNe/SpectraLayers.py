"""Spectra transformer encoder / decoder, MI355X build.

Same constructors, attributes and state_dict keys as the reference's
SpectraLayers.py; forward passes run on the HIP kernels.  The decoder's
982-token masked self-attention is the dominant cost of the whole step
(SURVEY.md §8(a) a7).
"""
import torch
from torch import nn

from . import _chain, _ops
from .util_layers import (MLP, Linear, SinusoidalMLPPositionalEmbedding,
                          SinusoidalPositionalEmbedding, TransformerBlock, decoder_fusable,
                          decoder_inputs, decoder_stack, decoder_stack_first,
                          singlelayerMLP, encoder_stack_steps)


class spectraTransformerDecoder(nn.Module):
    """SpectraLayers.py:11-63.  Queries sinMLP(wavelength); context =
    [contextfc(z) | sinMLP(phase)] (latent_len + 1 tokens); 4 blocks of masked
    self-attention + cross-attention; head 32->32->1."""

    def __init__(self, bottleneck_dim, model_dim=32, num_heads=4, ff_dim=32, num_layers=4,
                 dropout=0.1, selfattn=False):
        super().__init__()
        self.transformerblocks = nn.ModuleList(
            [TransformerBlock(model_dim, num_heads, ff_dim, dropout, selfattn)
             for _ in range(num_layers)])
        self.wavelength_embd_layer = SinusoidalMLPPositionalEmbedding(model_dim)
        self.phase_embd_layer = SinusoidalMLPPositionalEmbedding(model_dim)
        self.contextfc = MLP(bottleneck_dim, model_dim, [model_dim])
        self.get_flux = singlelayerMLP(model_dim, 1)

    def forward(self, wavelength, phase, bottleneck, mask=None, repeat=1, prepared=None):
        """`repeat` > 1: wavelength holds the B distinct rows of the N = repeat * B
        sequences (the decoders' K-sample / two-latent expand, SpectraVAE.py:189-192):
        the embedding MLP runs on the B rows and is broadcast (its gradient is the
        sum over the copies), the rest of the decoder on N.  `prepared`: this call's
        prepare() result, computed ahead (photospecMMVAE.forward: beside the encoders)."""
        if prepared is None:
            prepared = self.prepare(wavelength, phase, mask, repeat, bottleneck.shape[1] + 1)
        x_res, x_qkv, x_out, rep, phase_embd, first = prepared
        bottleneck = _ops.cat([self.contextfc(bottleneck), phase_embd], dim=1)
        h = decoder_stack(self.transformerblocks, x_res, bottleneck, mask, x_qkv=x_qkv,
                          rep=rep, first=first)
        return self.get_flux(x_out, h).squeeze(-1)   # get_flux(x + h)

    def prepare(self, wavelength, phase, mask=None, repeat=1, lc=1):
        """The part of forward() that does not read the latents: the wavelength and
        phase embeddings and, on the fused path, block 1's in-projection and
        its masked self-attention (util_layers.decoder_stack_first).  lc: context tokens
        (latent_len + 1)."""
        x = self.wavelength_embd_layer(wavelength)
        phase_embd = self.phase_embd_layer(phase[:, None])
        # x feeds the first block twice and the head: one gradient sum (_ops.fanout)
        x_res, x_qkv, x_out, rep = decoder_inputs(x, repeat, self.transformerblocks, lc)
        first = None
        if x_res.dim() == 3 and decoder_fusable(self.transformerblocks, lc):
            first = decoder_stack_first(self.transformerblocks, x_res, mask, x_qkv, rep)
        return x_res, x_qkv, x_out, rep, phase_embd, first


class spectraTransformerEncoder(nn.Module):
    """SpectraLayers.py:66-138.  NB the argument order (wavelength, flux, ...):
    SpectraEnc passes (flux, wavelength, ...) into it (SpectraVAE.py:41-44), so
    flux_embd sees the wavelength grid and the sinusoidal embedding sees the
    flux.  That is the reference's behaviour and is kept."""

    def __init__(self, bottleneck_length, bottleneck_dim, model_dim, num_heads, num_layers,
                 ff_dim, dropout=0.1, selfattn=False, concat=True):
        super().__init__()
        self.initbottleneck = nn.Parameter(torch.randn(bottleneck_length, model_dim))
        self.flux_embd = Linear(1, model_dim)
        self.transformerblocks = nn.ModuleList(
            [TransformerBlock(model_dim, num_heads, ff_dim, dropout, selfattn)
             for _ in range(num_layers)])
        self.bottleneckfc = singlelayerMLP(model_dim, bottleneck_dim)
        self.concat = concat
        if concat:
            self.spectrafc = MLP(2 * model_dim, model_dim, [model_dim])
            self.wavelength_embd_layer = SinusoidalPositionalEmbedding(model_dim)
        else:
            self.spectrafc = None
            self.wavelength_embd_layer = SinusoidalMLPPositionalEmbedding(model_dim)
        self.phase_embd_layer = SinusoidalMLPPositionalEmbedding(model_dim)

    def forward(self, wavelength, flux, phase, mask=None):
        return _chain.drive([self.steps(wavelength, flux, phase, mask)])[0]

    def steps(self, wavelength, flux, phase, mask=None):
        """forward as a generator (VAESNe._chain.drive), see photometricTransformerEncoder."""
        if self.concat:
            flux_embd = self.spectrafc(_ops.cat([self.flux_embd(flux[:, :, None]),
                                                  self.wavelength_embd_layer(wavelength)], dim=-1))
        else:
            flux_embd = self.flux_embd(flux[:, :, None],
                                       base=self.wavelength_embd_layer(wavelength))
        phase_embd = self.phase_embd_layer(phase[:, None])
        context = _ops.cat([flux_embd, phase_embd], dim=1)
        if mask is not None:
            # the phase token is never masked (SpectraLayers.py:129-131)
            mask = _ops.cat([mask, torch.zeros(mask.shape[0], 1, dtype=mask.dtype,
                                                device=mask.device)], dim=1)
        x = _ops.repeat_batch(self.initbottleneck, context.shape[0])
        x_res, x_qkv, x_out = _ops.fanout(x, 3)
        h = yield from encoder_stack_steps(self.transformerblocks, x_res, context,
                                           context_mask=mask, x_qkv=x_qkv)
        return self.bottleneckfc(x_out, h)   # bottleneckfc(x + h)
