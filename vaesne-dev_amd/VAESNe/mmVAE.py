"""Mixture-of-experts multimodal VAE over (light curve, spectrum) pairs,
MI355X build (reference: mmVAE.py:71-132, photospecMMVAE)."""
import torch
import torch.distributions as dist
import torch.nn as nn

from . import _ops


class _CellMatrix(list):
    """The 2x2 px_zs list of lists; `merged` holds the per-decoder (loc, scale)
    [K, 2B, L_d] tensors its cells are views of (empty if decoded per cell)."""

    def __init__(self, rows):
        super().__init__(rows)
        self.merged = []


class photospecMMVAE(nn.Module):
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
        qz_xs, zss = [], []
        for m, vae in enumerate(self.vaes):
            qz_x, zs = vae.posterior(x[m], K=K)
            qz_xs.append(qz_x)
            zss.append(zs)
        px_zs = _CellMatrix([[None for _ in range(n)] for _ in range(n)])
        if all(z.shape == zss[0].shape for z in zss):
            B = zss[0].shape[1]
            zcat = torch.cat(zss, dim=1)
            for d, vae in enumerate(self.vaes):
                loc, scale = vae.decode_params(zcat, x[d], groups=n)
                px_zs.merged.append((loc, scale))
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
