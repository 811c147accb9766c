"""Photometry (light-curve) transformer encoder / decoder, MI355X build.

Same constructors, attributes and state_dict keys as the reference's
PhotometricLayers.py; forward passes run on the HIP kernels.
"""
import torch
from torch import nn

from . import _chain, _ops
from .util_layers import (MLP, Linear, SinusoidalMLPPositionalEmbedding,
                          SinusoidalPositionalEmbedding, TransformerBlock, decoder_fusable,
                          decoder_inputs, decoder_stack, decoder_stack_first,
                          singlelayerMLP, encoder_stack_steps)


class photometricTransformerDecoder(nn.Module):
    """PhotometricLayers.py:10-69.  Queries are sinMLP(time) + band embedding;
    4 blocks of masked self-attention over the light-curve points and
    cross-attention to the decoded latent tokens; head 32->32->1."""

    def __init__(self, bottleneck_dim, num_bands, model_dim=32, num_heads=4, ff_dim=32,
                 num_layers=4, dropout=0.1, donotmask=False, selfattn=False):
        super().__init__()
        self.transformerblocks = nn.ModuleList(
            [TransformerBlock(model_dim, num_heads, ff_dim, dropout, selfattn)
             for _ in range(num_layers)])
        self.model_dim = model_dim
        self.sinusoidal_time_embd = SinusoidalMLPPositionalEmbedding(model_dim)
        self.bandembd = nn.Embedding(num_bands, model_dim)
        self.contextfc = MLP(bottleneck_dim, model_dim, [model_dim])
        self.get_photo = singlelayerMLP(model_dim, 1)
        self.donotmask = donotmask

    def forward(self, time, band, bottleneck, mask=None, repeat=1, prepared=None):
        """`repeat` > 1: time / band hold the B distinct rows of the N = repeat * B
        sequences (PhotometricVAE.py:190-193 expand): the embedding runs on the B rows
        and is broadcast (its gradient summed over the copies).  `prepared`: this
        call's prepare() result, computed ahead."""
        if self.donotmask:
            mask = None
        if prepared is None:
            prepared = self.prepare(time, band, mask, repeat, bottleneck.shape[1])
        x_res, x_qkv, x_out, rep, first = prepared
        bottleneck = self.contextfc(bottleneck)
        h = decoder_stack(self.transformerblocks, x_res, bottleneck, mask, x_qkv=x_qkv, rep=rep,
                          first=first)
        return self.get_photo(x_out, h).squeeze(-1)   # get_photo(x + h)

    def prepare(self, time, band, mask=None, repeat=1, lc=1):
        """The part of forward() that does not read the latents: the time / band
        embedding and, on the fused path, block 1's in-projection and
        its masked self-attention.  lc: context tokens (latent_len)."""
        if self.donotmask:
            mask = None
        # x = time_embd + band_embd (PhotometricLayers.py:62-64), the add fused in the gather
        x = _ops.embedding(band, self.bandembd.weight, base=self.sinusoidal_time_embd(time))
        # x feeds the first block twice and the head: one gradient sum (_ops.fanout)
        x_res, x_qkv, x_out, rep = decoder_inputs(x, repeat, self.transformerblocks, lc)
        first = None
        if x_res.dim() == 3 and decoder_fusable(self.transformerblocks, lc):
            first = decoder_stack_first(self.transformerblocks, x_res, mask, x_qkv, rep)
        return x_res, x_qkv, x_out, rep, first


class photometricTransformerEncoder(nn.Module):
    """PhotometricLayers.py:72-143.  Light-curve tokens (flux, time, band),
    2*latent_len learned query tokens cross-attending to them (key padding
    mask), bottleneck MLP."""

    def __init__(self, num_bands, bottleneck_length, bottleneck_dim, model_dim=32, num_heads=4,
                 ff_dim=32, num_layers=4, dropout=0.1, selfattn=False, concat=True):
        super().__init__()
        self.model_dim = model_dim
        self.initbottleneck = nn.Parameter(torch.randn(bottleneck_length, model_dim))
        self.bottleneckfc = singlelayerMLP(model_dim, bottleneck_dim)
        self.transformerblocks = nn.ModuleList(
            [TransformerBlock(model_dim, num_heads, ff_dim, dropout, selfattn)
             for _ in range(num_layers)])
        self.concat = concat
        self.bandembd = nn.Embedding(num_bands, model_dim)
        self.fluxfc = Linear(1, model_dim)
        if concat:
            self.time_embd = SinusoidalMLPPositionalEmbedding(model_dim)
            self.LCfc = MLP(3 * model_dim, model_dim, [model_dim])
        else:
            self.time_embd = SinusoidalPositionalEmbedding(model_dim)
            self.LCfc = None

    def forward(self, flux, time, band, mask=None):
        return _chain.drive([self.steps(flux, time, band, mask)])[0]

    def steps(self, flux, time, band, mask=None):
        """forward as a generator (VAESNe._chain.drive): yields the fused latent chain's
        work item so several encoders' chains can share one launch."""
        if self.concat:
            tok = self.LCfc(_ops.cat([self.fluxfc(flux[:, :, None]),
                                       self.time_embd(time),
                                       _ops.embedding(band, self.bandembd.weight)], dim=-1))
        else:
            # fluxfc(flux) + sin(time) + bandembd(band): both adds fused into the kernels
            tok = _ops.embedding(band, self.bandembd.weight,
                                 base=self.fluxfc(flux[:, :, None], base=self.time_embd(time)))
        x = _ops.repeat_batch(self.initbottleneck, flux.shape[0])
        x_res, x_qkv, x_out = _ops.fanout(x, 3)
        h = yield from encoder_stack_steps(self.transformerblocks, x_res, tok, context_mask=mask,
                                           x_qkv=x_qkv)
        return self.bottleneckfc(x_out, h)   # bottleneckfc(x + h)
