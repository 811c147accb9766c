"""Objectives, MI355X build (reference: losses.py).

Same functions and signatures as the reference; the log-probability / KL /
log-mean-exp arithmetic runs in fused HIP kernels reading the tensors of the
Laplace objects the models return:

    elbo(model, x, K=1, debug=False)   losses.py:16-24   (mean over K*B)
    _m_iwae(model, x, K=1) -> lw       losses.py:47-62   ([2K, B])
    m_iwae(model, x, K=1)              losses.py:78-93   (sum over B)
    compute_microbatch_split           losses.py:68-76
    negInfoNCE(model, x, temperature)  losses.py:98-110  (contrastive pretraining)
"""
import numpy as np
import torch

from . import _ops
from . import distributed as D


def expand_first_dim(t, K):
    shape = t.shape
    return t.unsqueeze(0).expand((K,) + shape)


def _pz(model):
    p = model.pz_params
    return p[0], p[1]


def elbo(model, x, K=1, debug=False):
    """E_{p(x)}[ELBO]: mean_{k,b}(llik * sum_L log p(x|z)) - mean_b sum KL(q(z|x) || p(z))."""
    qz_x, px_z, _ = model(x, K)
    if px_z.loc.device.type == "cpu":
        return _elbo_host(model, x, K, qz_x, px_z, debug)
    pz_loc, pz_scale = _pz(model)
    loss = _ops.ElboFn.apply(x[0], float(model.llik_scaling), px_z.loc, px_z.scale, qz_x.loc,
                             qz_x.scale, pz_loc, pz_scale)
    if debug:
        print(f"elbo: {loss.item()}")
    return loss


def _elbo_host(model, x, K, qz_x, px_z, debug=False):
    """elbo on host tensors — only the host-path image VAE (ImageVAE.HostImgVAE, BASELINE
    config 1) produces those; every HIP model refuses host
    tensors before reaching here.  losses.py:16-24 with torch's Laplace log_prob and
    closed-form KL (torch/distributions/kl.py:331-338)."""
    data = expand_first_dim(x[0], K)
    lpx = px_z.log_prob(data).reshape(*px_z.batch_shape[:2], -1) * model.llik_scaling
    kld = torch.distributions.kl_divergence(qz_x, model.pz(*model.pz_params))
    if debug:
        print(f"kl: {kld.sum((-1, -2)).mean()}, llk: {-lpx.sum(-1).mean()}")
    # a non-finite value is returned as the reference does; training_step raises on
    # it on every rank together (a raise here would be rank-local)
    return (lpx.sum(-1) - kld.sum((-1, -2))[None, :]).mean()


def _m_iwae(model, x, K=1):
    """IWAE log-weights for the 2-modality MoE VAE -> lw [2*K, B]."""
    if len(model.vaes) != 2:
        raise NotImplementedError("fused m_iwae covers the reference's two-modality photospecMMVAE")
    qz_xs, px_zs, zss = model(x, K)
    pz_loc, pz_scale = _pz(model)
    llik = [float(model.vaes[0].llik_scaling), float(model.vaes[1].llik_scaling)]
    merged = getattr(px_zs, "merged", None)
    if merged and _cells_are_views(px_zs, merged):
        (l0, s0), (l1, s1) = merged
        return _ops.IwaeLwMergedFn.apply(
            x[0][0], x[1][0], llik, l0, l1, s0, s1, zss[0], zss[1],
            qz_xs[0].loc, qz_xs[0].scale, qz_xs[1].loc, qz_xs[1].scale, pz_loc, pz_scale)
    return _ops.IwaeLwFn.apply(
        x[0][0], x[1][0], llik,
        px_zs[0][0].loc, px_zs[0][1].loc, px_zs[1][0].loc, px_zs[1][1].loc,
        px_zs[0][0].scale, px_zs[0][1].scale, px_zs[1][0].scale, px_zs[1][1].scale,
        zss[0], zss[1], qz_xs[0].loc, qz_xs[0].scale, qz_xs[1].loc, qz_xs[1].scale,
        pz_loc, pz_scale)


def _cells_are_views(px_zs, merged):
    """True iff every cell px_zs[e][d] still is the batch slice [eB, (e+1)B)
    of decoder d's merged (loc, scale) (a caller may have replaced cells)."""
    for d, (loc, scale) in enumerate(merged):
        B = loc.shape[1] // 2
        for e in range(2):
            c = px_zs[e][d]
            for t, full in ((c.loc, loc), (c.scale, scale)):
                if (t.data_ptr() != full.data_ptr() + e * B * full.stride(1) * full.element_size()
                        or t.shape != (full.shape[0], B, full.shape[2])
                        or t.stride() != full.stride()):
                    return False
    return True


def is_multidata(dataB):
    return isinstance(dataB, list)


def compute_microbatch_split(x, K):
    """losses.py:68-76 (a memory heuristic of the reference; never splits at
    realistic batch sizes)."""
    B = x[0][0].size(0) if is_multidata(x) else x[0].size(0)
    S = sum([1.0 / (K * np.prod(_x[0].size()[1:])) for _x in x]) if is_multidata(x) \
        else 1.0 / (K * np.prod(x[0].size()[1:]))
    S = int(1e8 * S)
    assert (S > 0), "Cannot fit individual data in memory, consider smaller K"
    return min(B, S)


def m_iwae(model, x, K=1):
    """IWAE estimate of log p(x) for the multimodal VAE: sum_b LME_{2K} lw."""
    S = compute_microbatch_split(x, K)
    n_chunk = len(x[0][0].split(S))
    lw = []
    for i in range(n_chunk):
        split_i = tuple(tuple(tensor.split(S)[i] for tensor in tensor_tuple) for tensor_tuple in x)
        lw.append(_m_iwae(model, split_i, K))
    lw = lw[0] if len(lw) == 1 else _ops.cat(lw, 1)
    return _ops.LmeSumFn.apply(lw)


### contrastive loss ###
def negInfoNCE(model, x, temperature=0.07):
    """Negative symmetric InfoNCE of the model's two projections (losses.py:98-110):
    -(CE(z1n z2n^T / T, arange) + CE(its transpose, arange)) / 2, one fused HIP
    kernel chain (normalise -> row/column log-sum-exp -> mean) that never
    materialises the B x B logits in HBM.  It couples every sample of the batch:
    under torch.distributed each rank passes its batch shard, the projections are
    all-gathered (distributed.global_rows) and each rank returns the full-batch
    value / world, so training_step's SUM gradient all-reduce (its multimodal
    default) gives the full-batch gradient and its logged loss the full value."""
    z1, z2 = model(x)
    z1, z2, scale = D.global_rows(z1, z2)
    loss = _ops.InfoNCEFn.apply(z1, z2, temperature)
    return loss if scale == 1.0 else loss * scale
