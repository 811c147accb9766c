"""ORACLE — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Functional CPU restatement of the reference's training step.  Parameters are a
flat ``{state_dict key: tensor}`` mapping that uses the reference's key layout,
so the same dict can be loaded into the reference modules (fixture generation)
and into the HIP build's modules (parity tests).  Every function cites the
reference file:line whose arithmetic it restates; paths are relative to
``/root/reference/package/VAESNe`` unless prefixed ``torch/`` (the installed
PyTorch 2.10 sources, which own the third-party arithmetic: MHA, Laplace, KL).

Precision: runs in whatever dtype the inputs/params carry (fp32 to match the
reference bit-for-bit-ish, fp64 as a high-precision judge for the GPU path).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

Params = Dict[str, torch.Tensor]


# ----------------------------------------------------------------------------
# configuration (mirrors the constructor kwargs the cannon scripts pass)
# ----------------------------------------------------------------------------
@dataclass
class VaeCfg:
    """One modality's VAE.  ``kind`` is 'photo' or 'spec'.

    Photometry defaults: PhotometricVAE.py:98-113; spectra: SpectraVAE.py:91-104.
    """
    kind: str
    latent_len: int = 4
    latent_dim: int = 4
    model_dim: int = 32
    num_heads: int = 4
    ff_dim: int = 32
    num_layers: int = 4
    selfattn: bool = False
    concat: bool = True
    beta: float = 1.0
    num_bands: int = 6          # photometry only
    llik_scaling: Optional[float] = None   # set by the MMVAE (mmVAE.py:82-84)
    bright: bool = False        # BrightPhotometricVAE / BrightSpectraVAE (concat=True encoders)

    def llik(self) -> float:
        return (1.0 / self.beta) if self.llik_scaling is None else self.llik_scaling


@dataclass
class MMVAECfg:
    """photospecMMVAE(vaes=[photo, spec], beta, length_ratio) — mmVAE.py:72-84."""
    photo: VaeCfg
    spec: VaeCfg
    beta: float = 1.0
    length_ratio: float = 982 / 60

    def __post_init__(self):
        # mmVAE.py:82-84: both 1/beta, photometry additionally * length_ratio
        self.photo.llik_scaling = (1.0 / self.beta)
        self.photo.llik_scaling *= self.length_ratio
        self.spec.llik_scaling = 1.0 / self.beta


# ----------------------------------------------------------------------------
# L1 building blocks (util_layers.py)
# ----------------------------------------------------------------------------
def _lin(p: Params, pre: str, x: torch.Tensor) -> torch.Tensor:
    """nn.Linear: y = x W^T + b."""
    return F.linear(x, p[pre + ".weight"], p[pre + ".bias"])


def single_layer_mlp(p: Params, pre: str, x):
    """singlelayerMLP: fc2(relu(fc1(x))) — util_layers.py:9-18."""
    return _lin(p, pre + ".fc2", torch.relu(_lin(p, pre + ".fc1", x)))


def mlp_one_hidden(p: Params, pre: str, x):
    """MLP(in, out, [hidden]) = Linear -> ReLU -> Linear — util_layers.py:20-34
    (Sequential indices 0 and 2)."""
    return _lin(p, pre + ".mlp.2", torch.relu(_lin(p, pre + ".mlp.0", x)))


def div_term_mlp(dim: int) -> torch.Tensor:
    """util_layers.py:138 — exp(arange(dim) * (-log(1e4)/dim)), fp32 recipe."""
    return torch.exp(torch.arange(0, dim).float() * (-torch.log(torch.tensor(10000.0)) / dim))


def div_term_plain(dim: int) -> torch.Tensor:
    """util_layers.py:122 — exp(arange(0,dim,2) * (-log(1e4)/dim))."""
    return torch.exp(torch.arange(0, dim, 2).float() * (-torch.log(torch.tensor(10000.0)) / dim))


def sinus_features(x: torch.Tensor, div: torch.Tensor) -> torch.Tensor:
    """[sin(x*d) | cos(x*d)] over the last (new) axis — util_layers.py:127-129, 144-146."""
    arg = x[..., None] * div.to(x.dtype)
    return torch.cat([torch.sin(arg), torch.cos(arg)], dim=-1)


def sinus_mlp_embed(p: Params, pre: str, x: torch.Tensor, dim: int) -> torch.Tensor:
    """SinusoidalMLPPositionalEmbedding.forward — util_layers.py:142-149."""
    e = sinus_features(x, div_term_mlp(dim))
    return _lin(p, pre + ".fc2", torch.relu(_lin(p, pre + ".fc1", e)))


def sinus_plain_embed(x: torch.Tensor, dim: int) -> torch.Tensor:
    """SinusoidalPositionalEmbedding.forward — util_layers.py:125-129 (no params)."""
    return sinus_features(x, div_term_plain(dim))


def _dropout(x, p_drop: float, training: bool):
    return F.dropout(x, p_drop, training) if (training and p_drop > 0) else x


def multihead_attention(p: Params, pre: str, xq, xkv, key_padding_mask, num_heads: int,
                        p_drop: float = 0.0, training: bool = False):
    """nn.MultiheadAttention(batch_first=True) slow path, restated:
    torch/nn/functional.py:6206 (in-projection with the packed [3E,E] weight),
    :6559-6594 (q scaled by 1/sqrt(head_dim) *before* QK^T; bool key padding
    mask -> -inf added to the scores; softmax; dropout on the probabilities;
    P V), then out_proj.  The head-averaged weights the reference also computes
    (:6606) are discarded by every caller (util_layers.py:289,297,301)."""
    W = p[pre + ".in_proj_weight"]
    b = p[pre + ".in_proj_bias"]
    E = W.shape[1]
    dh = E // num_heads
    q = F.linear(xq, W[:E], b[:E])
    k = F.linear(xkv, W[E:2 * E], b[E:2 * E])
    v = F.linear(xkv, W[2 * E:], b[2 * E:])
    Bn, Lq, _ = q.shape
    Lk = k.shape[1]
    q = q.view(Bn, Lq, num_heads, dh).transpose(1, 2) * math.sqrt(1.0 / float(dh))
    k = k.view(Bn, Lk, num_heads, dh).transpose(1, 2)
    v = v.view(Bn, Lk, num_heads, dh).transpose(1, 2)
    s = q @ k.transpose(-1, -2)                     # [B, H, Lq, Lk]
    if key_padding_mask is not None:
        s = s.masked_fill(key_padding_mask[:, None, None, :], float("-inf"))
    a = torch.softmax(s, dim=-1)
    a = _dropout(a, p_drop, training)
    o = (a @ v).transpose(1, 2).reshape(Bn, Lq, E)
    return _lin(p, pre + ".out_proj", o)


def layer_norm(p: Params, pre: str, x):
    """nn.LayerNorm(eps=1e-5) over the last axis."""
    return F.layer_norm(x, (x.shape[-1],), p[pre + ".weight"], p[pre + ".bias"], 1e-5)


def transformer_block(p: Params, pre: str, x, context=None, mask=None, context_mask=None,
                      num_heads: int = 4, p_drop: float = 0.0, training: bool = False):
    """TransformerBlock.forward — util_layers.py:285-309 (post-LN).
    The optional context self-attention exists iff its params exist (:269-274);
    its output is local to this block (:296-299)."""
    a = multihead_attention(p, pre + ".self_attn", x, x, mask, num_heads, p_drop, training)
    x = layer_norm(p, pre + ".layernorm1", x + _dropout(a, p_drop, training))
    if context is not None:
        if (pre + ".context_self_attn.in_proj_weight") in p:
            c = multihead_attention(p, pre + ".context_self_attn", context, context,
                                    context_mask, num_heads, p_drop, training)
            context = layer_norm(p, pre + ".layernorm_context", context + _dropout(c, p_drop, training))
        a = multihead_attention(p, pre + ".cross_attn", x, context, context_mask, num_heads,
                                p_drop, training)
        x = layer_norm(p, pre + ".layernorm2", x + _dropout(a, p_drop, training))
    f = _lin(p, pre + ".ffn.2", F.gelu(_lin(p, pre + ".ffn.0", x)))
    return layer_norm(p, pre + ".layernorm3", x + _dropout(f, p_drop, training))


def log_mean_exp(value: torch.Tensor, dim: int = 0) -> torch.Tensor:
    """util_layers.py:326-327."""
    return torch.logsumexp(value, dim) - math.log(value.size(dim))


# ----------------------------------------------------------------------------
# L2 modality networks (PhotometricLayers.py, SpectraLayers.py)
# ----------------------------------------------------------------------------
def photo_encoder(p: Params, pre: str, c: VaeCfg, flux, time, band, mask, p_drop, training):
    """photometricTransformerEncoder.forward — PhotometricLayers.py:117-143."""
    E = c.model_dim
    if c.concat:   # :127-130
        tok = torch.cat([_lin(p, pre + ".fluxfc", flux[:, :, None]),
                         sinus_mlp_embed(p, pre + ".time_embd", time, E),
                         p[pre + ".bandembd.weight"][band]], dim=-1)
        ctx = mlp_one_hidden(p, pre + ".LCfc", tok)
    else:          # :133-135
        ctx = (_lin(p, pre + ".fluxfc", flux[:, :, None]) + sinus_plain_embed(time, E)
               + p[pre + ".bandembd.weight"][band])
    x = p[pre + ".initbottleneck"][None].expand(flux.shape[0], -1, -1)   # :137-138
    h = x
    for i in range(c.num_layers):   # :140-142 (latent tokens unmasked, context masked)
        h = transformer_block(p, f"{pre}.transformerblocks.{i}", h, ctx, None, mask,
                              c.num_heads, p_drop, training)
    return single_layer_mlp(p, pre + ".bottleneckfc", x + h)            # :143


def photo_decoder(p: Params, pre: str, c: VaeCfg, time, band, z, mask, p_drop, training):
    """photometricTransformerDecoder.forward — PhotometricLayers.py:49-69."""
    x = sinus_mlp_embed(p, pre + ".sinusoidal_time_embd", time, c.model_dim) \
        + p[pre + ".bandembd.weight"][band]
    h = x
    ctx = mlp_one_hidden(p, pre + ".contextfc", z)
    for i in range(c.num_layers):   # self-attn masked, cross-attn unmasked (:66-67)
        h = transformer_block(p, f"{pre}.transformerblocks.{i}", h, ctx, mask, None,
                              c.num_heads, p_drop, training)
    return single_layer_mlp(p, pre + ".get_photo", x + h).squeeze(-1)


def spec_encoder(p: Params, pre: str, c: VaeCfg, flux, wavelength, phase, mask, p_drop, training):
    """spectraTransformerEncoder.forward — SpectraLayers.py:112-138.

    NB: SpectraEnc.forward (SpectraVAE.py:41-44) passes (flux, wavelength, ...)
    into the (wavelength, flux, ...) slots, so the Linear(1->E) 'flux_embd'
    sees the *wavelength* and the sinusoidal embedding sees the *flux*.  That
    swap is the reference's behaviour and is reproduced here."""
    E = c.model_dim
    arg_wavelength, arg_flux = flux, wavelength      # the swap
    if c.concat:   # :266-267
        tok = mlp_one_hidden(p, pre + ".spectrafc",
                             torch.cat([_lin(p, pre + ".flux_embd", arg_flux[:, :, None]),
                                        sinus_plain_embed(arg_wavelength, E)], dim=-1))
    else:
        tok = (_lin(p, pre + ".flux_embd", arg_flux[:, :, None])
               + sinus_mlp_embed(p, pre + ".wavelength_embd_layer", arg_wavelength, E))
    ph = sinus_mlp_embed(p, pre + ".phase_embd_layer", phase[:, None], E)   # :271
    ctx = torch.cat([tok, ph], dim=1)                                       # :272
    if mask is not None:                                                    # :273-275
        mask = torch.cat([mask, torch.zeros(mask.shape[0], 1, dtype=torch.bool)], dim=1)
    x = p[pre + ".initbottleneck"][None].expand(ctx.shape[0], -1, -1)
    h = x
    for i in range(c.num_layers):
        h = transformer_block(p, f"{pre}.transformerblocks.{i}", h, ctx, None, mask,
                              c.num_heads, p_drop, training)
    return single_layer_mlp(p, pre + ".bottleneckfc", x + h)


def spec_decoder(p: Params, pre: str, c: VaeCfg, wavelength, phase, z, mask, p_drop, training):
    """spectraTransformerDecoder.forward — SpectraLayers.py:46-63."""
    E = c.model_dim
    x = sinus_mlp_embed(p, pre + ".wavelength_embd_layer", wavelength, E)
    ph = sinus_mlp_embed(p, pre + ".phase_embd_layer", phase[:, None], E)
    ctx = torch.cat([mlp_one_hidden(p, pre + ".contextfc", z), ph], dim=1)   # [N, Lz+1, E]
    h = x
    for i in range(c.num_layers):
        h = transformer_block(p, f"{pre}.transformerblocks.{i}", h, ctx, mask, None,
                              c.num_heads, p_drop, training)
    return single_layer_mlp(p, pre + ".get_flux", x + h).squeeze(-1)


# ----------------------------------------------------------------------------
# L3 VAEs
# ----------------------------------------------------------------------------
@dataclass
class Laplace:
    """The (loc, scale) pair of a torch.distributions.Laplace."""
    loc: torch.Tensor
    scale: torch.Tensor

    def log_prob(self, v):
        """torch/distributions/laplace.py:88-91."""
        return -torch.log(2 * self.scale) - torch.abs(v - self.loc) / self.scale


def laplace_rsample(loc, scale, u):
    """torch/distributions/laplace.py:74-86 with the uniform draw u ~ U(eps-1, 1)
    supplied by the caller (the reference draws it with loc.new(shape).uniform_)."""
    return loc - scale * u.sign() * torch.log1p(-u.abs())


def draw_u(shape, dtype=torch.float32, generator=None):
    """The reference's draw: loc.new(shape).uniform_(eps - 1, 1) (laplace.py:83)."""
    eps = torch.finfo(dtype).eps
    return torch.empty(shape, dtype=dtype).uniform_(eps - 1, 1, generator=generator)


def encode(p: Params, pre: str, c: VaeCfg, x, p_drop=0.0, training=False):
    """PhotometricEnc.forward (PhotometricVAE.py:41-56) / SpectraEnc.forward
    (SpectraVAE.py:40-51): mu = b[:, :Lz], scale = softplus(b[:, Lz:])."""
    if c.kind == "photo":
        flux, time, band, mask = x
        b = photo_encoder(p, pre + "enc.inference_transformer", c, flux, time, band, mask,
                          p_drop, training)
    else:
        flux, wavelength, phase, mask = x
        b = spec_encoder(p, pre + "enc.inference_transformer", c, flux, wavelength, phase, mask,
                         p_drop, training)
    return b[:, :c.latent_len, :], F.softplus(b[:, c.latent_len:, :])


def decode(p: Params, pre: str, c: VaeCfg, zs, x, p_drop=0.0, training=False) -> Laplace:
    """PhotometricVAE.decode (:188-199) + PhotometricDec.forward (:89-94):
    scale = 1 + 1e8*mask;  SpectraVAE.decode (:186-196) + SpectraDec.forward
    (:82-87): scale = 1 + 1e10*mask.  The data are expanded K times."""
    K = zs.shape[0]
    zf = zs.reshape(-1, zs.shape[-2], zs.shape[-1])
    if c.kind == "photo":
        _, time, band, mask = x
        L = time.shape[1]
        rep = lambda t: t.unsqueeze(0).expand(K, -1, -1).reshape(-1, L)
        loc = photo_decoder(p, pre + "dec.generativetransformer", c, rep(time), rep(band), zf,
                            rep(mask), p_drop, training)
        big = 1e8
    else:
        _, wavelength, phase, mask = x
        L = wavelength.shape[1]
        rep = lambda t: t.unsqueeze(0).expand(K, -1, -1).reshape(-1, L)
        loc = spec_decoder(p, pre + "dec.generativetransformer", c, rep(wavelength),
                           phase.unsqueeze(0).expand(K, -1).reshape(-1), zf, rep(mask),
                           p_drop, training)
        big = 1e10
    m = rep(mask)
    scale = torch.ones_like(loc)
    scale = scale + big * m
    loc = loc.reshape(K, -1, L)
    if c.bright:
        # BrightPhotometricVAE.decode (PhotometricVAE.py:321-329) / BrightSpectraVAE.decode
        # (SpectraVAE.py:311-319): brightnessfc(first latent token [| phase]) replaces the
        # decoded curve's mean over L.
        inp = zs[:, :, 0, :]
        if c.kind == "spec":
            inp = torch.cat((inp, phase.unsqueeze(0).expand(K, -1)[:, :, None]), dim=-1)
        brightness = mlp_one_hidden(p, pre + "brightnessfc", inp)
        loc = loc + brightness - loc.mean(axis=2)[:, :, None]
    return Laplace(loc, scale.reshape(K, -1, L))


def vae_forward(p, pre, c: VaeCfg, x, K, u, p_drop=0.0, training=False):
    """PhotometricVAE.forward (:157-176) / SpectraVAE.forward (:148-165)."""
    mu, scale = encode(p, pre, c, x, p_drop, training)
    zs = laplace_rsample(mu, scale, u)
    return Laplace(mu, scale), decode(p, pre, c, zs, x, p_drop, training), zs


def mmvae_forward(p, cfg: MMVAECfg, x, K, us, p_drop=0.0, training=False):
    """photospecMMVAE.forward — mmVAE.py:91-106: diagonal cells from each VAE's
    forward, off-diagonal px_zs[e][d] = vae_d.decode(zs_e, x[d])."""
    cfgs = [cfg.photo, cfg.spec]
    qz, zss = [], []
    px = [[None, None], [None, None]]
    for m in range(2):
        q, pxz, zs = vae_forward(p, f"vaes.{m}.", cfgs[m], x[m], K, us[m], p_drop, training)
        qz.append(q)
        zss.append(zs)
        px[m][m] = pxz
    for e in range(2):
        for d in range(2):
            if e != d:
                px[e][d] = decode(p, f"vaes.{d}.", cfgs[d], zss[e], x[d], p_drop, training)
    return qz, px, zss


def mmvae_generate(p, cfg: MMVAECfg, x, N, u):
    """photospecMMVAE.generate -- mmVAE.py:108-118: latents = Laplace(_pz_params)
    .rsample([N, B]) (u [N, B, Lz, Dz]), decoded by every modality at its x grid; the
    decoders' means (= loc).  Eval mode: no dropout."""
    z = laplace_rsample(p["_pz_params.0"], p["_pz_params.1"], u)
    cfgs = [cfg.photo, cfg.spec]
    return [decode(p, f"vaes.{d}.", cfgs[d], z, x[d]).loc for d in range(2)]


def spectra_generate(p, pre: str, c: VaeCfg, x, N, u):
    """SpectraVAE.generate -- SpectraVAE.py:198-206: zs = Laplace(pz_params).rsample(
    [N, 1]) (u [N, 1, Lz, Dz]) decoded at x's grid (one conditioning spectrum: the
    reference's decode expands x K = N times against N latent rows), returned as
    mean.unsqueeze(0) [1, N, 1, L]."""
    z = laplace_rsample(p[pre + "_pz_params.0"], p[pre + "_pz_params.1"], u)
    return decode(p, pre, c, z, x).loc.unsqueeze(0)


# ----------------------------------------------------------------------------
# L5 objectives (losses.py)
# ----------------------------------------------------------------------------
def _m_iwae(p, cfg: MMVAECfg, x, K, us, p_drop=0.0, training=False):
    """losses.py:47-62 -> lw [2K, B]."""
    qz, px, zss = mmvae_forward(p, cfg, x, K, us, p_drop, training)
    cfgs = [cfg.photo, cfg.spec]
    pz = Laplace(p["_pz_params.0"], p["_pz_params.1"])
    lws = []
    for r in range(2):
        lpz = pz.log_prob(zss[r]).sum([-1, -2])
        lqz = log_mean_exp(torch.stack([q.log_prob(zss[r]).sum([-1, -2]) for q in qz]))
        lpx = torch.stack([px[r][d].log_prob(x[d][0]).view(*px[r][d].loc.shape[:2], -1)
                           .mul(cfgs[d].llik()).sum(-1) for d in range(2)]).sum(0)
        lws.append(lpz + lpx - lqz)
    return torch.cat(lws), (qz, px, zss)


def compute_microbatch_split(x, K):
    """losses.py:68-76 (never splits at realistic batch sizes)."""
    B = x[0][0].size(0)
    S = sum(1.0 / (K * math.prod(_x[0].size()[1:])) for _x in x)
    S = int(1e8 * S)
    assert S > 0
    return min(B, S)


def m_iwae(p, cfg: MMVAECfg, x, K, us, p_drop=0.0, training=False):
    """losses.py:78-93: LME over the 2K importance samples, summed over batch.
    ``us`` is the pair of noise draws for the whole batch; chunks slice it."""
    S = compute_microbatch_split(x, K)
    B = x[0][0].size(0)
    lw, aux = [], None
    for s0 in range(0, B, S):
        xs = [tuple(t[s0:s0 + S] for t in m) for m in x]
        us_i = [u[:, s0:s0 + S] for u in us]
        l, aux = _m_iwae(p, cfg, xs, K, us_i, p_drop, training)
        lw.append(l)
    lw = torch.cat(lw, 1)
    return log_mean_exp(lw).sum(), lw, aux


def kl_laplace_std(q: Laplace):
    """kl_divergence(q, Laplace(0,1)) via torch/distributions/kl.py:331-338."""
    ratio = q.scale / 1.0
    ad = (q.loc - 0.0).abs()
    return -ratio.log() + ad / 1.0 + ratio * torch.exp(-ad / q.scale) - 1


def elbo(p, c: VaeCfg, x, K, u, p_drop=0.0, training=False):
    """losses.py:16-24 — mean over (K, B) of llik*sum_L log p(x|z) - sum KL."""
    q, pxz, zs = vae_forward(p, "", c, x, K, u, p_drop, training)
    data = x[0].unsqueeze(0).expand((K,) + x[0].shape)
    lpx = pxz.log_prob(data).reshape(*pxz.loc.shape[:2], -1) * c.llik()
    kld = kl_laplace_std(q)
    return (lpx.sum(-1) - kld.sum((-1, -2))[None, :]).mean(), (q, pxz, zs)


# ----------------------------------------------------------------------------
# optimizer: torch.optim.AdamW defaults (the scripts construct AdamW(params, lr))
# ----------------------------------------------------------------------------
@dataclass
class AdamWState:
    lr: float = 1e-3
    betas: Tuple[float, float] = (0.9, 0.999)
    eps: float = 1e-8
    weight_decay: float = 1e-2
    step: int = 0
    m: Dict[str, torch.Tensor] = field(default_factory=dict)
    v: Dict[str, torch.Tensor] = field(default_factory=dict)


def adamw_step(p: Params, grads: Dict[str, torch.Tensor], st: AdamWState):
    """torch/optim/adamw.py single-tensor update (decoupled weight decay,
    bias-corrected first/second moments)."""
    st.step += 1
    b1, b2 = st.betas
    bc1 = 1 - b1 ** st.step
    bc2 = 1 - b2 ** st.step
    with torch.no_grad():
        for k, g in grads.items():
            if g is None:
                continue
            w = p[k]
            if k not in st.m:
                st.m[k] = torch.zeros_like(w)
                st.v[k] = torch.zeros_like(w)
            w.mul_(1 - st.lr * st.weight_decay)
            st.m[k].lerp_(g, 1 - b1)
            st.v[k].mul_(b2).addcmul_(g, g, value=1 - b2)
            denom = (st.v[k].sqrt() / math.sqrt(bc2)).add_(st.eps)
            w.addcdiv_(st.m[k], denom, value=-(st.lr / bc1))


# ----------------------------------------------------------------------------
# contrastive pretraining + regression heads (§8(f) row 4)
# ----------------------------------------------------------------------------
@dataclass
class ContrastCfg:
    """ContraPhotSpec(...) kwargs — contrastiveNets.py:24-46 (concat=True encoders)."""
    latent_len: int = 4
    latent_dim: int = 4
    proj_dim: int = 8
    num_bands: int = 6
    photo_model_dim: int = 32
    photo_num_heads: int = 4
    photo_ff_dim: int = 32
    photo_num_layers: int = 4
    spec_model_dim: int = 32
    spec_num_heads: int = 4
    spec_num_layers: int = 4
    spec_ff_dim: int = 32
    selfattn: bool = False

    def photo(self) -> VaeCfg:
        return VaeCfg("photo", self.latent_len, self.latent_dim, self.photo_model_dim,
                      self.photo_num_heads, self.photo_ff_dim, self.photo_num_layers,
                      self.selfattn, True, 1.0, self.num_bands)

    def spec(self) -> VaeCfg:
        return VaeCfg("spec", self.latent_len, self.latent_dim, self.spec_model_dim,
                      self.spec_num_heads, self.spec_ff_dim, self.spec_num_layers,
                      self.selfattn, True)


def contrast_forward(p: Params, c: ContrastCfg, x, p_drop=0.0, training=False):
    """ContraPhotSpec.forward — contrastiveNets.py:74-85: both encoders (the spectra
    one with the reference's (flux, wavelength) slot swap), flatten, singlelayerMLP
    projections."""
    pf, pt, pb, pm = x[0]
    sf, sw, sp, sm = x[1]
    z1 = photo_encoder(p, "photometry_encoder", c.photo(), pf, pt, pb, pm, p_drop, training)
    z2 = spec_encoder(p, "spectra_encoder", c.spec(), sf, sw, sp, sm, p_drop, training)
    z1 = single_layer_mlp(p, "photo_proj", z1.reshape(z1.shape[0], -1))
    z2 = single_layer_mlp(p, "spectra_proj", z2.reshape(z2.shape[0], -1))
    return z1, z2


def neg_info_nce(z1, z2, temperature=0.07):
    """negInfoNCE — losses.py:98-110, with F.normalize (x / max(||x||, 1e-12),
    torch/nn/functional.py normalize) and cross_entropy(mean) written out."""
    n1 = z1 / z1.norm(dim=-1, keepdim=True).clamp_min(1e-12)
    n2 = z2 / z2.norm(dim=-1, keepdim=True).clamp_min(1e-12)
    logits = n1 @ n2.T / temperature
    diag = torch.diagonal(logits)
    ce_r = (torch.logsumexp(logits, dim=1) - diag).mean()
    ce_c = (torch.logsumexp(logits, dim=0) - diag).mean()
    return -(ce_r + ce_c) / 2


def mlp(p: Params, pre: str, x, n_hidden: int):
    """MLP(in, out, hidden) — util_layers.py:20-34: Linear/ReLU pairs at Sequential
    indices 0, 2, ..., final Linear at 2*n_hidden."""
    for i in range(n_hidden):
        x = torch.relu(_lin(p, f"{pre}.mlp.{2 * i}", x))
    return _lin(p, f"{pre}.mlp.{2 * n_hidden}", x)


def end2end_regression(p: Params, kind: str, c: VaeCfg, x, n_hidden: int, p_drop=0.0,
                       training=False):
    """photoend2endregression / specend2endregression.forward — regression.py:100-105,
    137-141: encoder -> flatten -> MLP."""
    enc = photo_encoder if kind == "photo" else spec_encoder
    h = enc(p, "enc", c, *x, p_drop, training)
    return mlp(p, "outfc", h.reshape(h.shape[0], -1), n_hidden)


def encoder_param_shapes(c: VaeCfg, prefix: str) -> Dict[str, Tuple[int, ...]]:
    """The bare encoder module's keys (contrastive / end-to-end nets build the
    encoder with latent_len query tokens, not the VAE's 2*latent_len)."""
    src = "enc.inference_transformer."
    out = {}
    for k, v in param_shapes(c).items():
        if k.startswith(src):
            kk = prefix + k[len(src):]
            out[kk] = (c.latent_len, c.model_dim) if kk.endswith("initbottleneck") else v
    return out


def contrast_param_shapes(c: ContrastCfg) -> Dict[str, Tuple[int, ...]]:
    s = encoder_param_shapes(c.photo(), "photometry_encoder.")
    s.update(encoder_param_shapes(c.spec(), "spectra_encoder."))
    n = c.latent_len * c.latent_dim
    for pre in ("photo_proj", "spectra_proj"):
        s[pre + ".fc1.weight"], s[pre + ".fc1.bias"] = (n, n), (n,)
        s[pre + ".fc2.weight"], s[pre + ".fc2.bias"] = (c.proj_dim, n), (c.proj_dim,)
    return s


# ----------------------------------------------------------------------------
# deterministic parameter construction (shared with tests/golden/gen_golden.py)
# ----------------------------------------------------------------------------
def _attn_keys(pre):
    return [pre + ".in_proj_weight", pre + ".in_proj_bias", pre + ".out_proj.weight",
            pre + ".out_proj.bias"]


def param_shapes(cfg, prefix: str = "") -> Dict[str, Tuple[int, ...]]:
    """state_dict key -> shape for a VaeCfg (prefix '' / 'vaes.{m}.') or an
    MMVAECfg.  Mirrors the reference module tree (used to build param dicts
    for the oracle without importing the reference)."""
    if isinstance(cfg, MMVAECfg):
        out = {"_pz_params.0": (cfg.photo.latent_len, cfg.photo.latent_dim),
               "_pz_params.1": (cfg.photo.latent_len, cfg.photo.latent_dim)}
        out.update(param_shapes(cfg.photo, "vaes.0."))
        out.update(param_shapes(cfg.spec, "vaes.1."))
        return out
    c: VaeCfg = cfg
    E, F_, Dz, Lz = c.model_dim, c.ff_dim, c.latent_dim, c.latent_len
    s: Dict[str, Tuple[int, ...]] = {}

    def lin(pre, i, o):
        s[pre + ".weight"] = (o, i)
        s[pre + ".bias"] = (o,)

    def block(pre, ctx_self):
        for a in (["self_attn", "cross_attn"] + (["context_self_attn"] if ctx_self else [])):
            s[f"{pre}.{a}.in_proj_weight"] = (3 * E, E)
            s[f"{pre}.{a}.in_proj_bias"] = (3 * E,)
            lin(f"{pre}.{a}.out_proj", E, E)
        if ctx_self:
            s[pre + ".layernorm_context.weight"] = (E,)
            s[pre + ".layernorm_context.bias"] = (E,)
        lin(pre + ".ffn.0", E, F_)
        lin(pre + ".ffn.2", F_, E)
        for n in ("layernorm1", "layernorm2", "layernorm3"):
            s[f"{pre}.{n}.weight"] = (E,)
            s[f"{pre}.{n}.bias"] = (E,)

    s[prefix + "_pz_params.0"] = (Lz, Dz)
    s[prefix + "_pz_params.1"] = (Lz, Dz)
    enc = prefix + "enc.inference_transformer"
    dec = prefix + "dec.generativetransformer"
    if c.kind == "photo":
        s[enc + ".initbottleneck"] = (2 * Lz, E)
        lin(enc + ".bottleneckfc.fc1", E, E)
        lin(enc + ".bottleneckfc.fc2", E, Dz)
        for i in range(c.num_layers):
            block(f"{enc}.transformerblocks.{i}", c.selfattn)
        s[enc + ".bandembd.weight"] = (c.num_bands, E)
        lin(enc + ".fluxfc", 1, E)
        if c.concat:
            lin(enc + ".time_embd.fc1", 2 * E, E)
            lin(enc + ".time_embd.fc2", E, E)
            lin(enc + ".LCfc.mlp.0", 3 * E, E)
            lin(enc + ".LCfc.mlp.2", E, E)
        for i in range(c.num_layers):
            block(f"{dec}.transformerblocks.{i}", False)
        lin(dec + ".sinusoidal_time_embd.fc1", 2 * E, E)
        lin(dec + ".sinusoidal_time_embd.fc2", E, E)
        s[dec + ".bandembd.weight"] = (c.num_bands, E)
        lin(dec + ".contextfc.mlp.0", Dz, E)
        lin(dec + ".contextfc.mlp.2", E, E)
        lin(dec + ".get_photo.fc1", E, E)
        lin(dec + ".get_photo.fc2", E, 1)
    else:
        s[enc + ".initbottleneck"] = (2 * Lz, E)
        lin(enc + ".flux_embd", 1, E)
        for i in range(c.num_layers):
            block(f"{enc}.transformerblocks.{i}", c.selfattn)
        lin(enc + ".bottleneckfc.fc1", E, E)
        lin(enc + ".bottleneckfc.fc2", E, Dz)
        if c.concat:
            lin(enc + ".spectrafc.mlp.0", 2 * E, E)
            lin(enc + ".spectrafc.mlp.2", E, E)
        else:
            lin(enc + ".wavelength_embd_layer.fc1", 2 * E, E)
            lin(enc + ".wavelength_embd_layer.fc2", E, E)
        lin(enc + ".phase_embd_layer.fc1", 2 * E, E)
        lin(enc + ".phase_embd_layer.fc2", E, E)
        for i in range(c.num_layers):
            block(f"{dec}.transformerblocks.{i}", False)
        lin(dec + ".wavelength_embd_layer.fc1", 2 * E, E)
        lin(dec + ".wavelength_embd_layer.fc2", E, E)
        lin(dec + ".phase_embd_layer.fc1", 2 * E, E)
        lin(dec + ".phase_embd_layer.fc2", E, E)
        lin(dec + ".contextfc.mlp.0", Dz, E)
        lin(dec + ".contextfc.mlp.2", E, E)
        lin(dec + ".get_flux.fc1", E, E)
        lin(dec + ".get_flux.fc2", E, 1)
    if c.bright:   # MLP(latent_dim [+ 1 phase], 1, [model_dim]): PhotometricVAE.py:284, SpectraVAE.py:268
        lin(prefix + "brightnessfc.mlp.0", Dz + (1 if c.kind == "spec" else 0), E)
        lin(prefix + "brightnessfc.mlp.2", E, 1)
    return s


def make_params(cfg, fill, dtype=torch.float32, requires_grad=False) -> Params:
    """Build a param dict with ``fill(key, shape) -> np.ndarray | None``
    (None = keep the reference's constant init: _pz_params zeros/ones)."""
    out: Params = {}
    shapes = cfg if isinstance(cfg, dict) else (
        contrast_param_shapes(cfg) if isinstance(cfg, ContrastCfg) else param_shapes(cfg))
    for k, shp in shapes.items():
        v = fill(k, shp)
        if v is None:
            t = torch.zeros(shp) if k.endswith("_pz_params.0") else torch.ones(shp)
            out[k] = t.to(dtype)
        else:
            out[k] = torch.as_tensor(v).to(dtype).reshape(shp)
            if requires_grad:
                out[k].requires_grad_(True)
    return out


def trainable_keys(p: Params) -> List[str]:
    return [k for k in p if "_pz_params" not in k]
