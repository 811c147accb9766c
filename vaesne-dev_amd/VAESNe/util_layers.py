"""Building blocks of the VAESNe transformer stacks, MI355X build.

Mirrors the hot-path symbols of the reference's util_layers.py (same class
names, constructor signatures, attribute and state_dict names) so checkpoints'
state_dicts and the cannon scripts keep working:

    singlelayerMLP            util_layers.py:9-18
    MLP                       util_layers.py:20-34
    SinusoidalPositionalEmbedding     :113-129
    SinusoidalMLPPositionalEmbedding  :131-149
    TransformerBlock          util_layers.py:257-309
    get_mean / log_mean_exp / kl_divergence   :313-336

Forward passes run on the HIP kernels (VAESNe._ops); there is no CPU path.
"""
from __future__ import annotations

import contextlib
import math

import torch
from torch import nn

from . import _chain, _config, _ops


class Linear(nn.Linear):
    """nn.Linear whose forward runs on the HIP linear kernel."""

    def forward(self, x, act=None, x2=None, base=None):
        return _ops.linear(x, self.weight, self.bias, act=act, x2=x2, base=base)


class ReferencePickle:
    """Mixin of the top-level models: a whole-module pickle written by the REFERENCE
    (torch.save(model), cannon/test_spectra.py:94, loaded by torch.load in
    cannon/try_spectra_model.py:29 and the other try_* / test/goldstein scripts)
    unpickles into this package's classes by module path; its leaf layers are plain
    torch nn.Linear / nn.MultiheadAttention.  After unpickling they are re-classed to
    the HIP Linear / MultiheadAttention (same parameters, same state), so the loaded
    model runs on the HIP path (tests/test_pickle_compat.py, tests/test_gpu_parity.py)."""

    def __setstate__(self, state):
        super().__setstate__(state)
        upgrade_reference_modules(self)


def upgrade_reference_modules(root):
    """Re-class torch nn.Linear / nn.MultiheadAttention leaves of `root` (in place)."""
    for m in root.modules():
        t = type(m)
        if t is nn.Linear:
            m.__class__ = Linear
        elif t is nn.MultiheadAttention:
            m.__class__ = MultiheadAttention
    return root


########### simple MLPs ###############
class singlelayerMLP(nn.Module):
    """fc2(relu(fc1(x))) — util_layers.py:9-18.  `x2` (optional) is added to x
    inside the first kernel (the reference's `f(x + h)` residual calls)."""

    def __init__(self, in_dim, out_dim):
        super().__init__()
        self.fc1 = Linear(in_dim, in_dim)
        self.fc2 = Linear(in_dim, out_dim)

    def forward(self, x, x2=None):
        if _ops.mlp_head_ok(x, self.fc1, self.fc2):     # E -> 1 heads: one fused kernel
            return _ops.mlp_head(x, x2, self.fc1, self.fc2)
        return self.fc2(self.fc1(x, act="relu", x2=x2))


class MLP(nn.Module):
    """Linear -> ReLU -> ... -> Linear — util_layers.py:20-34 (keys mlp.0, mlp.2, ...)."""

    def __init__(self, in_dim, out_dim, hidden_dim=[64, 64]):
        super().__init__()
        layers = []
        for i in range(len(hidden_dim)):
            layers.append(Linear(in_dim if i == 0 else hidden_dim[i - 1], hidden_dim[i]))
            layers.append(nn.ReLU())
        layers.append(Linear(hidden_dim[-1], out_dim))
        self.mlp = nn.Sequential(*layers)

    def forward(self, x):
        mods = list(self.mlp)
        for i in range(0, len(mods) - 1, 2):
            x = mods[i](x, act="relu")
        return mods[-1](x)


################# positional encoding ###################
class _DivTerm:
    """The reference's div_term, computed on the host exactly as the reference
    (fp32 torch ops), cached per device (the reference re-copies it H2D on every
    call, util_layers.py:127,144)."""

    def __init__(self, t: torch.Tensor):
        self.cpu = t
        self._dev = {}

    def on(self, device):
        key = str(device)
        d = self._dev.get(key)
        if d is None:
            d = self.cpu.to(device)
            self._dev[key] = d
        return d

    def __getstate__(self):
        return {"cpu": self.cpu}

    def __setstate__(self, state):
        self.cpu, self._dev = state["cpu"], {}


def _restore_div(module, state):
    """A reference pickle holds the tensor `div_term` (util_layers.py:122,138)."""
    div = state.pop("div_term", None)
    nn.Module.__setstate__(module, state)
    if div is not None and "_div" not in module.__dict__:
        module._div = _DivTerm(div.float().cpu())


class SinusoidalPositionalEmbedding(nn.Module):
    """[sin(x*d), cos(x*d)] with d = exp(arange(0,dim,2) * -ln(1e4)/dim) — util_layers.py:113-129."""

    def __init__(self, dim=64):
        super().__init__()
        self.dim = dim
        self._div = _DivTerm(torch.exp(torch.arange(0, dim, 2).float() *
                                       (-torch.log(torch.tensor(10000.0)) / dim)))

    def __setstate__(self, state):
        _restore_div(self, state)

    @property
    def div_term(self):
        return self._div.cpu

    def forward(self, x):
        return _ops.sincos(x, self._div.on(x.device))


class SinusoidalMLPPositionalEmbedding(nn.Module):
    """sin/cos over d = exp(arange(dim) * -ln(1e4)/dim), then fc2(relu(fc1(.)))
    — util_layers.py:131-149."""

    def __init__(self, dim=64):
        super().__init__()
        self.dim = dim
        self._div = _DivTerm(torch.exp(torch.arange(0, dim).float() *
                                       (-torch.log(torch.tensor(10000.0)) / dim)))
        self.fc1 = Linear(2 * dim, dim)
        self.fc2 = Linear(dim, dim)

    def __setstate__(self, state):
        _restore_div(self, state)

    @property
    def div_term(self):
        return self._div.cpu

    def forward(self, x):
        enc = _ops.sincos(x, self._div.on(x.device))
        return self.fc2(self.fc1(enc, act="relu"))


################# attention ###################
class MultiheadAttention(nn.MultiheadAttention):
    """nn.MultiheadAttention (same parameters, init and state_dict keys) whose
    forward runs the fused HIP path: packed in-projection kernel, flash-style
    masked attention kernel (dropout on the probabilities in train mode), then
    the out-projection kernel.  Returns (output, None): the reference discards
    the head-averaged weights at every call site (util_layers.py:289,297,301)."""

    def forward(self, query, key, value, key_padding_mask=None, need_weights=True,
                attn_mask=None, average_attn_weights=True, is_causal=False):
        if attn_mask is not None or is_causal:
            raise NotImplementedError("VAESNe attention: attn_mask / is_causal are not used by the reference")
        if not self.batch_first:
            raise NotImplementedError("VAESNe attention is batch_first (as the reference)")
        if key is not value:
            raise NotImplementedError("VAESNe attention expects key is value")
        E, H = self.embed_dim, self.num_heads
        p = self.dropout if self.training else 0.0
        W, b = self.in_proj_weight, self.in_proj_bias
        if query is key:
            qkv = _ops.linear(query, W, b)
            o = _ops.self_attention(qkv, key_padding_mask, H, p)
        else:
            q, kv = _ops.in_proj_pair(query, key, W, b)
            o = _ops.cross_attention(q, kv, key_padding_mask, H, p)
        return _ops.linear(o, self.out_proj.weight, self.out_proj.bias), None


class TransformerBlock(nn.Module):
    """Post-LN block with optional context self-attention and cross-attention
    — util_layers.py:257-309.  Each residual join is one fused
    residual+dropout+LayerNorm kernel; the FFN is Linear+GELU fused, Linear."""

    def __init__(self, embed_dim, num_heads, ff_dim, dropout=0.1, context_self_attn=False):
        super().__init__()
        self.self_attn = MultiheadAttention(embed_dim, num_heads, dropout=dropout, batch_first=True)
        self.cross_attn = MultiheadAttention(embed_dim, num_heads, dropout=dropout, batch_first=True)
        if context_self_attn:
            self.context_self_attn = MultiheadAttention(embed_dim, num_heads, dropout=dropout,
                                                        batch_first=True)
            self.layernorm_context = nn.LayerNorm(embed_dim)
        else:
            self.context_self_attn = None
        self.ffn = nn.Sequential(
            Linear(embed_dim, ff_dim),
            nn.GELU(),
            Linear(ff_dim, embed_dim),
        )
        self.layernorm1 = nn.LayerNorm(embed_dim)
        self.layernorm2 = nn.LayerNorm(embed_dim)
        self.layernorm3 = nn.LayerNorm(embed_dim)
        self.dropout = nn.Dropout(dropout)

    def forward(self, x, context=None, mask=None, context_mask=None):
        p = self.dropout.p if self.training else 0.0
        a, _ = self.self_attn(x, x, x, key_padding_mask=mask)
        x = _ops.add_layernorm(x, a, self.layernorm1, p)
        if context is not None:
            if self.context_self_attn is not None:
                c, _ = self.context_self_attn(context, context, context, key_padding_mask=context_mask)
                context = _ops.add_layernorm(context, c, self.layernorm_context, p)
            a, _ = self.cross_attn(x, context, context, key_padding_mask=context_mask)
            x = _ops.add_layernorm(x, a, self.layernorm2, p)
        f = self.ffn[2](self.ffn[0](x, act="gelu"))
        return _ops.add_layernorm(x, f, self.layernorm3, p)


def _fusable_decoder_block(blk):
    E = blk.layernorm1.normalized_shape[0]
    return (blk.context_self_attn is None and E == 32 and blk.self_attn.num_heads == 4
            and blk.cross_attn.num_heads == 4 and blk.ffn[0].out_features == 32
            and abs(blk.cross_attn.dropout - blk.dropout.p) < 1e-12
            and all(ln.eps == 1e-5 for ln in (blk.layernorm1, blk.layernorm2, blk.layernorm3)))


def decoder_fusable(blocks, context):
    """Whether decoder_stack runs these blocks as fused kernels (else per op).
    `context`: the context tensor [N, Lc, E], or its token count Lc."""
    blocks = list(blocks)
    if isinstance(context, torch.Tensor):
        if context.dim() != 3:
            return False
        context = context.shape[1]
    return bool(blocks) and all(_fusable_decoder_block(b) for b in blocks) and context <= 8


def decoder_inputs(xd, repeat, blocks, context):
    """The decoders' input embedding xd [Bd, L, E] of the distinct sequences, used by
    N = repeat * Bd sequences (the K samples x latents expand) -> (x_res, x_qkv, x_out,
    rep) for decoder_stack(x_res, ..., x_qkv=x_qkv, rep=rep) and the output head.
    Every use is an alias whose gradients one kernel sums (_ops.fanout); on the fused
    path the first in-projection reads the distinct rows (rep = repeat).
    `context`: the decoder's context tensor or its token count."""
    if repeat > 1 and decoder_fusable(blocks, context):
        xd_qkv, xd_rep = _ops.fanout(xd, 2)
        x = _ops.repeat_batch(xd_rep, repeat).reshape(repeat * xd.shape[0], *xd.shape[1:])
        x_res, x_out = _ops.fanout(x, 2)
        return x_res, xd_qkv, x_out, repeat
    x = xd
    if repeat > 1:
        x = _ops.repeat_batch(xd, repeat).reshape(repeat * xd.shape[0], *xd.shape[1:])
    x_res, x_qkv, x_out = _ops.fanout(x, 3)
    return x_res, x_qkv, x_out, 1


class DecoderFirst:
    """What a fused decoder stack computes before it needs the context: block 1's
    in-projection and masked self-attention read only the decoder input (the
    embedding of the wavelength / time grid, SpectraLayers.py:54-62,
    PhotometricLayers.py:59-67), not the latents, so they run while the encoders
    still work (photospecMMVAE.forward issues them on the photometry stream)."""
    __slots__ = ("N", "L", "kbias", "O1")

    def __init__(self, N, L, kbias, O1):
        self.N, self.L, self.kbias, self.O1 = N, L, kbias, O1

    def tensors(self):
        return [t for t in (self.kbias, self.O1) if t is not None]


def decoder_stack_first(blocks, x, mask=None, x_qkv=None, rep=1):
    """Block 1's in-projection and masked self-attention of a fused decoder stack
    (see decoder_stack): -> DecoderFirst."""
    blocks = list(blocks)
    E = 32
    L = x.shape[1]
    N = x.shape[0]
    b0 = blocks[0].self_attn
    p_attn = b0.dropout if blocks[0].training else 0.0
    qkv = _ops.linear(x if x_qkv is None else x_qkv, b0.in_proj_weight, b0.in_proj_bias)
    kbias = _ops.key_bias(mask)          # one mask conversion for all layers
    if rep > 1 and _ops.rep_attention_ok(qkv, b0.num_heads, rep):
        Bd = N // rep
        kb = None if kbias is None else kbias[:Bd]
        O1 = _ops.self_attention_rep(qkv, kb, b0.num_heads, p_attn, rep)
    else:
        if rep > 1:
            qkv = _ops.repeat_batch(qkv, rep).reshape(N, L, 3 * E)
        O1 = _ops.self_attention(qkv, None, b0.num_heads, p_attn, kbias=kbias)
    return DecoderFirst(N, L, kbias, O1)


def decoder_stack(blocks, x, context, mask=None, x_qkv=None, rep=1, first=None):
    """`for blk in blocks: x = blk(x, context, mask=mask)` for the decoders
    (SpectraLayers.py:61-62, PhotometricLayers.py:66-67).  With the reference's
    decoder shape (E 32, 4 heads, ff 32, no context self-attention) each block
    runs as: masked self-attention kernel -> ONE fused tail kernel (out_proj,
    LN1, cross-attention over the context tokens, LN2, FFN, LN3, and the next
    block's in_proj).  Other shapes take the per-op path (TransformerBlock).
    `x_qkv` (optional): an alias of x (_ops.fanout) the first in-projection reads,
    so the caller's single gradient sum for x covers that use too.
    `rep` > 1: x holds rep copies of Bd = N / rep distinct sequences (row r*Bd + b)
    and x_qkv is the [Bd, L, E] distinct rows: the first block's in-projection and
    self-attention scores run once per distinct sequence (_ops.self_attention_rep;
    each copy keeps its own dropout masks); mask must be repeated the same way.
    `first`: block 1's in-projection and self-attention already computed
    (decoder_stack_first on the same x / mask / rep)."""
    blocks = list(blocks)
    if x.dim() != 3 or not decoder_fusable(blocks, context):
        if rep > 1 or first is not None:
            raise RuntimeError("decoder_stack(rep > 1 / first) needs the fused decoder blocks")
        for blk in blocks:
            x = blk(x, context, mask=mask)
        return x
    if first is None:
        first = decoder_stack_first(blocks, x, mask, x_qkv, rep)
    elif first.N != x.shape[0] or first.L != x.shape[1]:
        raise RuntimeError("decoder_stack: `first` was computed for another input")
    L, kbias = first.L, first.kbias
    # every block's cross-attention reads the context: one gradient sum for all
    ctxs = _ops.fanout(context, len(blocks))
    qkv = None
    for i, blk in enumerate(blocks):
        p_attn = blk.self_attn.dropout if blk.training else 0.0
        p = blk.dropout.p if blk.training else 0.0
        if i == 0:
            O = first.O1
        else:
            O = _ops.self_attention(qkv, None, blk.self_attn.num_heads, p_attn, kbias=kbias)
        nxt = blocks[i + 1].self_attn if i + 1 < len(blocks) else None
        x, qkv = _ops.DecTailFn.apply(
            L, p, x, O, ctxs[i], blk.cross_attn.in_proj_weight, blk.cross_attn.in_proj_bias,
            blk.self_attn.out_proj.weight, blk.self_attn.out_proj.bias,
            blk.layernorm1.weight, blk.layernorm1.bias,
            blk.cross_attn.out_proj.weight, blk.cross_attn.out_proj.bias,
            blk.layernorm2.weight, blk.layernorm2.bias,
            blk.ffn[0].weight, blk.ffn[0].bias, blk.ffn[2].weight, blk.ffn[2].bias,
            blk.layernorm3.weight, blk.layernorm3.bias,
            None if nxt is None else nxt.in_proj_weight, None if nxt is None else nxt.in_proj_bias)
    return x


_CTX_STREAMS = {}


def _ctx_stream(t, i=0):
    """The stream block i's context self-attention path runs on: VAESNE_CTX_STREAMS
    streams (default 2: A/B 12.43 vs 12.60 ms per step with 1, 12.59 with 4) shared
    round-robin, so in the backward (issued last) the paths run two at a time
    (_config.streams off: none)."""
    if not t.is_cuda or not _config.streams:
        return None
    dev = t.device.index if t.device.index is not None else torch.cuda.current_device()
    i %= _config.ctx_streams
    st = _CTX_STREAMS.setdefault(dev, {})
    if i not in st:
        st[i] = torch.cuda.Stream(device=dev)
    return st[i]


def _fusable_encoder_block(blk):
    E = blk.layernorm1.normalized_shape[0]
    return (E == 32 and blk.self_attn.num_heads == 4 and blk.cross_attn.num_heads == 4
            and blk.ffn[0].out_features == 32
            and all(ln.eps == 1e-5 for ln in (blk.layernorm1, blk.layernorm2, blk.layernorm3)))


def _context_paths(blocks, context, context_mask):
    """Per-block context paths (x = LN(c + Drop(SelfAttn(c))) of each block with a
    context self-attention; the plain context otherwise) -> (ctxs, events).
    Every block reads the ORIGINAL context (twice with a context self-attention:
    its in-projection and its residual): aliases whose gradients one kernel sums.
    The paths are independent of each other and of the latent chain, so they run
    ahead on their own streams, one event per block for the join."""
    uses = [2 if b.context_self_attn is not None else 1 for b in blocks]
    cal = iter(_ops.fanout(context, sum(uses)))
    cuse = [[next(cal) for _ in range(u)] for u in uses]
    ctxs = [cu[0] for cu in cuse]
    evs = [None] * len(blocks)
    if not any(b.context_self_attn is not None for b in blocks):
        return ctxs, evs
    main = torch.cuda.current_stream() if _ctx_stream(context) is not None else None
    kb = _ops.key_bias_of(context_mask)     # built on the main stream, shared by all paths
    for i, blk in enumerate(blocks):
        if blk.context_self_attn is None:
            continue
        cs = _ctx_stream(context, i)
        if cs is not None:
            cs.wait_stream(main)
            # tensors crossing streams are recorded on their consumer stream, so the
            # caching allocator never hands their memory to the producer stream while
            # the consumer may still read it (the B=16 step read a reused block as
            # block i's context in the k|v weight gradient without this)
            _ops.used_on(cs, context, *cuse[i], kb)
        p = blk.dropout.p if blk.training else 0.0
        c_in, c_res = cuse[i]
        with torch.cuda.stream(cs) if cs is not None else contextlib.nullcontext():
            c, _ = blk.context_self_attn(c_in, c_in, c_in, key_padding_mask=context_mask)
            ctxs[i] = _ops.add_layernorm(c_res, c, blk.layernorm_context, p)
            if cs is not None:
                evs[i] = torch.cuda.Event()
                evs[i].record(cs)
                _ops.used_on(main, ctxs[i])
    return ctxs, evs


def _mergeable_context_paths(blocks, context):
    if len(blocks) < 2 or not _config.ctx_merge:
        return False
    m0 = blocks[0].context_self_attn
    if m0 is None or context.dim() != 3:
        return False
    for b in blocks:
        m = b.context_self_attn
        if (m is None or m.num_heads != m0.num_heads or m.dropout != m0.dropout
                or m.in_proj_bias is None or m.out_proj.bias is None
                or not m.batch_first or m.embed_dim != context.shape[-1]):
            return False
    return True


def _merged_context_paths(blocks, context, context_mask):
    """The G blocks' context paths as one batch-stacked path: the G in-projections
    write [G, B, L, 3E] (GroupLinearFn), ONE attention launch runs all G*B
    sequences (G x the workgroups of a per-block launch, which at B=16 x 983 tokens
    fills half the chip at best), the G out-projections read their slices back,
    then each block's residual + LayerNorm.  Per block the arithmetic is the
    per-block path's (util_layers.py:297-298); only the dropout draws come from one
    RNG call instead of G.  One stream, one event for the join."""
    G = len(blocks)
    B, L, E = context.shape
    mhas = [b.context_self_attn for b in blocks]
    H = mhas[0].num_heads
    pa = mhas[0].dropout if blocks[0].training else 0.0
    cal = _ops.fanout(context, 1 + G)      # the in-projections' input + G residuals
    cs = _ctx_stream(context, 0)
    main = torch.cuda.current_stream() if cs is not None else None
    kb = _ops.key_bias_rep(context_mask, G)
    if cs is not None:
        cs.wait_stream(main)
        _ops.used_on(cs, context, *cal, kb)
    ev = None
    with torch.cuda.stream(cs) if cs is not None else contextlib.nullcontext():
        qkv = _ops.group_linear(cal[0], [m.in_proj_weight for m in mhas],
                                [m.in_proj_bias for m in mhas], shared=True)
        o = _ops.self_attention(qkv.view(G * B, L, 3 * E), None, H, pa, kbias=kb)
        cs_ = _ops.group_linear(o.view(G, B, L, E), [m.out_proj.weight for m in mhas],
                                [m.out_proj.bias for m in mhas], shared=False)
        ctxs = [_ops.add_layernorm(cal[1 + i], cs_[i], blk.layernorm_context,
                                   blk.dropout.p if blk.training else 0.0)
                for i, blk in enumerate(blocks)]
        if cs is not None:
            ev = torch.cuda.Event()
            ev.record(cs)
            _ops.used_on(main, *ctxs)
    return ctxs, [ev] + [None] * (G - 1)


def encoder_stack(blocks, x, context, context_mask=None, x_qkv=None):
    """`for blk in blocks: x = blk(x, context, context_mask=context_mask)` for the
    encoders (SpectraLayers.py:135-136, PhotometricLayers.py:141-143: unmasked
    latent tokens x, the ORIGINAL data tokens as every block's context).  With the
    reference's shape the latent side of all blocks is ONE fused chain launch
    (VAESNe._chain; _config.enc_chain off selects the per-block path: latent
    self-attention core -> PRE (out_proj, LN1, cross q) + context k|v projection ->
    cross-attention core -> POST (out_proj, LN2, FFN, LN3, next in_proj)).  The
    optional context self-attention (spectra `selfattn`) runs ahead of the latent
    chain: batch-stacked over the blocks (_merged_context_paths) or per block."""
    return _chain.drive([encoder_stack_steps(blocks, x, context, context_mask, x_qkv)])[0]


def encoder_stack_steps(blocks, x, context, context_mask=None, x_qkv=None):
    """encoder_stack as a generator (VAESNe._chain.drive): runs everything up to the
    fused latent chain, yields the chain's work item (or None when the blocks take
    the per-op path), receives the chain output and returns it.  Driving several
    encoders' generators together launches their chains as ONE kernel."""
    blocks = list(blocks)
    if not blocks or not all(_fusable_encoder_block(b) for b in blocks) or x.dim() != 3:
        yield None
        for blk in blocks:
            x = blk(x, context, context_mask=context_mask)
        return x
    chain = _chain.fusable(blocks, x) and _config.enc_chain
    if chain and not any(b.context_self_attn is not None for b in blocks):
        # every block reads the original context: one input, its gradient summed in the op
        spec = _chain.make_spec(blocks, context_mask, shared=True)
        return (yield (spec, x, [context], blocks))
    if _mergeable_context_paths(blocks, context):
        ctxs, evs = _merged_context_paths(blocks, context, context_mask)
    else:
        ctxs, evs = _context_paths(blocks, context, context_mask)
    if chain:
        for ev in evs:
            if ev is not None:
                torch.cuda.current_stream().wait_event(ev)
        spec = _chain.make_spec(blocks, context_mask, shared=False)
        return (yield (spec, x, ctxs, blocks))
    yield None
    return _encoder_stack_ops(blocks, x, context_mask, x_qkv, ctxs, evs)


def _encoder_stack_ops(blocks, x, context_mask, x_qkv, ctxs, evs):
    """The per-block encoder path (PRE / cross-attention / POST launches)."""
    b0 = blocks[0].self_attn
    qkv = _ops.linear(x if x_qkv is None else x_qkv, b0.in_proj_weight, b0.in_proj_bias)
    for i, blk in enumerate(blocks):
        p = blk.dropout.p if blk.training else 0.0
        pa = blk.self_attn.dropout if blk.training else 0.0
        pc = blk.cross_attn.dropout if blk.training else 0.0
        O = _ops.self_attention(qkv, None, blk.self_attn.num_heads, pa)
        ctx = ctxs[i]
        if evs[i] is not None:
            torch.cuda.current_stream().wait_event(evs[i])

        x1, q, kv = _ops.EncPreFn.apply(
            p, x, O, ctx, blk.self_attn.out_proj.weight, blk.self_attn.out_proj.bias,
            blk.layernorm1.weight, blk.layernorm1.bias,
            blk.cross_attn.in_proj_weight, blk.cross_attn.in_proj_bias)
        c = _ops.cross_attention(q, kv, context_mask, blk.cross_attn.num_heads, pc)
        nxt = blocks[i + 1].self_attn if i + 1 < len(blocks) else None
        x, qkv = _ops.EncPostFn.apply(
            p, x1, c, blk.cross_attn.out_proj.weight, blk.cross_attn.out_proj.bias,
            blk.layernorm2.weight, blk.layernorm2.bias,
            blk.ffn[0].weight, blk.ffn[0].bias, blk.ffn[2].weight, blk.ffn[2].bias,
            blk.layernorm3.weight, blk.layernorm3.bias,
            None if nxt is None else nxt.in_proj_weight, None if nxt is None else nxt.in_proj_bias)
    return x


############## vae use ###################
def get_mean(d, K=100):
    """util_layers.py:313-323."""
    try:
        mean = d.mean
    except NotImplementedError:
        samples = d.rsample(torch.Size([K]))
        mean = samples.mean(0)
    return mean


def log_mean_exp(value, dim=0, keepdim=False):
    """util_layers.py:326-327 (API utility; the fused objectives do not call it)."""
    return torch.logsumexp(value, dim, keepdim=keepdim) - math.log(value.size(dim))


def kl_divergence(d1, d2, K=100):
    """util_layers.py:330-336 (API utility; `losses.elbo` uses the fused kernel)."""
    if (type(d1), type(d2)) in torch.distributions.kl._KL_REGISTRY:
        return torch.distributions.kl_divergence(d1, d2)
    samples = d1.rsample(torch.Size([K]))
    return (d1.log_prob(samples) - d2.log_prob(samples)).mean(0)
