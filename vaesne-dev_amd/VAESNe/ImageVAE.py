"""Host-galaxy image VAE — reference ImageVAE.py (HostImgEnc :9-54, HostImgDec
:56-107, HostImgVAE :110-242).

HOST (CPU) PATH for BASELINE config 1 (cannon/mnist.py: HostImgVAE + elbo +
training_step), SURVEY.md §8(a) a16 "CPU plumbing, no HIP kernel": every op is
PyTorch's own.  `losses.elbo` takes its host branch for these models
(losses._elbo_host).  A non-finite posterior raises RuntimeError where the
reference calls breakpoint() (ImageVAE.py:193-194).
"""
import torch
import torch.distributions as dist
import torch.nn.functional as F
from torch import nn

from .ImageLayers import (HostImgTransformerDecoder, HostImgTransformerDecoderHybrid,
                          HostImgTransformerEncoder)
from .base_vae import VAE


class HostImgEnc(nn.Module):
    """ImageVAE.py:9-54: bottleneck [B, 2*latent_len, latent_dim] -> (mu, softplus)."""

    def __init__(self, img_size, latent_len, latent_dim, patch_size=4, in_channels=3,
                 focal_loc=False, model_dim=32, num_heads=4, ff_dim=32, num_layers=4, dropout=0.1,
                 selfattn=False):
        super().__init__()
        self.inference_transformer = HostImgTransformerEncoder(
            img_size, 2 * latent_len, latent_dim, patch_size, in_channels, focal_loc, model_dim,
            num_heads, ff_dim, num_layers, dropout, selfattn)
        self.latent_dim = latent_dim
        self.latent_len = latent_len

    def forward(self, image, event_loc=None):
        b = self.inference_transformer(image, event_loc)
        return b[:, :self.latent_len, :], F.softplus(b[:, self.latent_len:, :])


class HostImgDec(nn.Module):
    """ImageVAE.py:56-107: (image loc, unit scale)."""

    def __init__(self, img_size, latent_dim, patch_size=4, in_channels=3, model_dim=32,
                 num_heads=4, ff_dim=32, num_layers=4, dropout=0.1, selfattn=False, hybrid=True):
        super().__init__()
        if hybrid:
            self.generativetransformer = HostImgTransformerDecoderHybrid(
                img_size, latent_dim, patch_size, in_channels, model_dim, num_heads, ff_dim,
                num_layers, dropout, selfattn)
        else:
            self.generativetransformer = HostImgTransformerDecoder(
                img_size, latent_dim, in_channels, model_dim, num_heads, ff_dim, num_layers,
                dropout, selfattn)

    def pxz(self, z):
        return self.generativetransformer(z)

    def forward(self, z):
        x_rec = self.pxz(z)
        return x_rec, torch.ones_like(x_rec)


class HostImgVAE(VAE):
    def __init__(self, img_size, latent_len, latent_dim, patch_size=4, in_channels=3,
                 focal_loc=False, model_dim=32, num_heads=4, ff_dim=32, num_layers=4, dropout=0.1,
                 selfattn=False, hybrid=True, beta=1., prior=dist.Laplace,
                 likelihood=dist.Laplace, posterior=dist.Laplace):
        super().__init__(
            prior, likelihood, posterior,
            HostImgEnc(img_size, latent_len, latent_dim, patch_size, in_channels, focal_loc,
                       model_dim, num_heads, ff_dim, num_layers, dropout, selfattn),
            HostImgDec(img_size, latent_dim, patch_size, in_channels, model_dim, num_heads, ff_dim,
                       num_layers, dropout, selfattn, hybrid),
            params=[img_size, latent_len, latent_dim, patch_size, in_channels, focal_loc,
                    model_dim, num_heads, ff_dim, num_layers, dropout, selfattn])
        self._pz_params = nn.ParameterList([
            nn.Parameter(torch.zeros(latent_len, latent_dim), requires_grad=False),
            nn.Parameter(torch.ones(latent_len, latent_dim), requires_grad=False),
        ])
        self.llik_scaling = 1. / beta
        self.modelName = 'HostImage'
        self.image_size = img_size
        self.in_channels = in_channels
        self.patch_size = patch_size
        self.latent_len = latent_len
        self.latent_dim = latent_dim
        self.focal_loc = focal_loc

    def _split(self, x):
        # training_step hands (image, label) batches; only focal_loc models use x[1]
        return (x[0], x[1]) if self.focal_loc else (x[0], None)

    def forward(self, x, K=1):
        """ImageVAE.py:187-198 -> (qz_x, px_z, zs)."""
        image, event_loc = self._split(x)
        self._qz_x_params = self.enc(image, event_loc)
        mu, scale = self._qz_x_params
        if not (torch.isfinite(mu).all() and torch.isfinite(scale).all()):
            raise RuntimeError("HostImgVAE: non-finite posterior location / scale (the reference "
                               "stops here, ImageVAE.py:193-194)")
        qz_x = self.qz_x(*self._qz_x_params)
        zs = qz_x.rsample(torch.Size([K]))
        return qz_x, self.decode(zs), zs

    def encode(self, x, mean=True):
        image, event_loc = self._split(x)
        self.eval()
        with torch.no_grad():
            qz_x = self.qz_x(*self.enc(image, event_loc))
        return qz_x.mean if mean else qz_x

    def decode(self, zs):
        """ImageVAE.py:213-220: px_z over [K, B, C, H, W]."""
        K = zs.shape[0]
        loc, scale = self.dec(zs.reshape(-1, zs.shape[-2], zs.shape[-1]))
        shape = (K, -1, self.in_channels, self.image_size, self.image_size)
        return self.px_z(loc.reshape(shape), scale.reshape(shape))

    def reconstruct(self, x, K=1):
        image, event_loc = self._split(x)
        self.eval()
        with torch.no_grad():
            qz_x = self.qz_x(*self.enc(image, event_loc))
            return self.decode(qz_x.rsample([K])).mean

    def generate(self, N):
        self.eval()
        with torch.no_grad():
            zs = self.pz(*self.pz_params).rsample(torch.Size([N]))
            return self.px_z(*self.dec(zs)).mean
