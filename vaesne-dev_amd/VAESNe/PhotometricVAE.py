"""Photometry VAE, MI355X build (reference: PhotometricVAE.py:10-355).

Encoder -> (mu, softplus scale) -> Laplace.rsample([K]) -> decoder, each step
a HIP kernel.  Constructors accept and ignore `photometric_length` (the
cannon scripts pass it).
"""
import torch
import torch.distributions as dist
from torch import nn

from . import _chain, _ops
from .PhotometricLayers import photometricTransformerDecoder, photometricTransformerEncoder
from .base_vae import VAE, check_laplace
from .util_layers import MLP, ReferencePickle


class PhotometricEnc(nn.Module):
    """PhotometricVAE.py:10-56: bottleneck [B, 2*latent_len, latent_dim] ->
    mu = b[:, :latent_len], scale = softplus(b[:, latent_len:])."""

    def __init__(self, num_bands, latent_len, latent_dim, model_dim, num_heads, ff_dim,
                 num_layers, dropout=0.1, selfattn=False, concat=True):
        super().__init__()
        self.inference_transformer = photometricTransformerEncoder(
            num_bands, 2 * latent_len, latent_dim, model_dim, num_heads, ff_dim, num_layers,
            dropout, selfattn, concat)
        self.latent_dim = latent_dim
        self.latent_len = latent_len

    def forward(self, flux, time, band, mask=None):
        return _chain.drive([self.steps(flux, time, band, mask)])[0]

    def steps(self, flux, time, band, mask=None):
        bottleneck = yield from self.inference_transformer.steps(flux, time, band, mask)
        return _ops.latent_head(bottleneck, self.latent_len)


class PhotometricDec(nn.Module):
    """PhotometricVAE.py:58-94: returns (loc, 1 + 1e8*mask)."""

    def __init__(self, latent_dim, num_bands, model_dim, num_heads, ff_dim, num_layers,
                 dropout=0.1, selfattn=False):
        super().__init__()
        self.generativetransformer = photometricTransformerDecoder(
            latent_dim, num_bands, model_dim, num_heads, ff_dim, num_layers, dropout, selfattn)

    def pxz(self, time, band, z, mask=None, repeat=1, prepared=None):
        return self.generativetransformer(time, band, z, mask, repeat=repeat, prepared=prepared)

    def forward(self, time, band, z, mask=None, repeat=1, prepared=None):
        x_rec = self.pxz(time, band, z, mask, repeat=repeat, prepared=prepared)
        if mask is None:
            var = torch.ones_like(x_rec)
        else:
            var = _ops.mask_scale(mask, 1, 1e8, x_rec).view_as(x_rec)
        return x_rec, var


class PhotometricVAE(ReferencePickle, VAE):
    def __init__(self, num_bands=6, latent_len=8, latent_dim=4, model_dim=64, num_heads=4,
                 ff_dim=64, num_layers=4, dropout=0.1, selfattn=False, concat=True, beta=1.,
                 prior=dist.Laplace, likelihood=dist.Laplace, posterior=dist.Laplace,
                 photometric_length=None):
        check_laplace(prior, likelihood, posterior)
        super().__init__(
            prior, likelihood, posterior,
            PhotometricEnc(num_bands, latent_len, latent_dim, model_dim, num_heads, ff_dim,
                           num_layers, dropout, selfattn, concat),
            PhotometricDec(latent_dim, num_bands, model_dim, num_heads, ff_dim, num_layers,
                           dropout),
            params=[num_bands, latent_len, latent_dim, model_dim, num_heads, ff_dim, num_layers,
                    dropout, selfattn])
        self._pz_params = nn.ParameterList([
            nn.Parameter(torch.zeros(latent_len, latent_dim), requires_grad=False),  # loc
            nn.Parameter(torch.ones(latent_len, latent_dim), requires_grad=False),   # scale
        ])
        self.llik_scaling = 1. / beta
        self.modelName = 'light_curve'
        self.latent_len = latent_len
        self.latent_dim = latent_dim

    def forward(self, x, K=1):
        """PhotometricVAE.py:157-176 -> (qz_x, px_z, zs)."""
        qz_x, zs = self.posterior(x, K)
        px_z = self.decode(zs, x)
        return qz_x, px_z, zs

    def posterior(self, x, K=1):
        """Encoder -> q(z|x) and K reparameterised draws (PhotometricVAE.py:158-163)."""
        return _chain.drive([self.posterior_steps(x, K)])[0]

    def posterior_steps(self, x, K=1):
        """posterior as a generator (VAESNe._chain.drive: several VAEs' encoder chains
        in one launch)."""
        params = yield from self.encoder_steps(x)
        return self.sample(params, K)

    def encoder_steps(self, x):
        """The encoder alone as a generator (-> (loc, scale) of q(z|x))."""
        flux, time, band, mask = x
        return (yield from self.enc.steps(flux, time, band, mask))

    def sample(self, params, K=1):
        """q(z|x) of the encoder output `params` and its K reparameterised draws."""
        # q(z|x) reads aliases of (loc, scale) whose gradients the sampler's backward adds
        z, *params = _ops.posterior_rsample(*params, K)
        self._qz_x_params = tuple(params)
        return self._dist(self.qz_x, *params), z

    def encode(self, x, mean=True):
        flux, time, band, mask = x
        self.eval()
        with torch.no_grad():
            qz_x = self._dist(self.qz_x, *self.enc(flux, time, band, mask))
        if mean:
            return qz_x.mean
        return qz_x

    def decode(self, zs, x):
        """PhotometricVAE.py:188-199: expand time/band/mask K times, decode,
        wrap in the likelihood distribution [K, B, L]."""
        return self._dist(self.px_z, *self.decode_params(zs, x))

    def _dec_mask(self, x, K, groups):
        mask = x[3]
        B, L = x[1].shape
        return None if mask is None else \
            mask.unsqueeze(0).unsqueeze(0).expand(K, groups, B, L).reshape(-1, L)

    def decode_prepare(self, x, K, groups=1):
        """The latent-independent part of decode_params(zs, x, groups) for K samples
        (embedding, block 1's in-projection and self-attention):
        -> `prepared` for decode_params."""
        _, time, band, _ = x
        mask = self._dec_mask(x, K, groups)
        return (K, groups, mask, self.dec.generativetransformer.prepare(
            time, band, mask, repeat=K * groups, lc=self.latent_len))

    def decode_params(self, zs, x, groups=1, prepared=None):
        """(loc, scale) [K, groups*B, L] for latents zs [K, groups*B, Lz, Dz]
        decoded at x's grid, x's batch repeated `groups` times (group-major).
        `prepared`: decode_prepare(x, K, groups) computed ahead."""
        _, time, band, _ = x
        K = zs.shape[0]
        B, L = time.shape
        if prepared is not None and prepared[:2] == (K, groups):
            mask, pre = prepared[2], prepared[3]
        else:
            mask, pre = self._dec_mask(x, K, groups), None
        # the time / band embedding runs once per distinct light curve (repeat = K * groups)
        loc, scale = self.dec(time, band, zs.reshape(-1, zs.shape[-2], zs.shape[-1]), mask,
                              repeat=K * groups, prepared=pre)
        return loc.reshape(K, groups * B, L), scale.reshape(K, groups * B, L)

    def reconstruct(self, x, K=1):
        self.eval()
        with torch.no_grad():
            mu, scale = self.enc(*x)
            zs = _ops.laplace_rsample(mu, scale, K)
            return self.decode(zs, x).mean

    def generate(self, N, time, band, mask=None):
        """Decode N prior draws at the given (time, band[, mask]) grid
        (the reference's version references an undefined K, PhotometricVAE.py:216)."""
        self.eval()
        with torch.no_grad():
            loc, scale = self.pz_params[0], self.pz_params[1]
            zs = _ops.laplace_rsample(loc.expand(time.shape[0], *loc.shape).contiguous(),
                                      scale.expand(time.shape[0], *scale.shape).contiguous(), N)
            return self.decode(zs, (None, time, band, mask)).mean


class BrightPhotometricVAE(PhotometricVAE):
    """PhotometricVAE.py:226-355: the first latent token carries the light curve's
    overall brightness.  decode() adds brightnessfc(zs[:, :, 0, :]) to the decoded
    curve after removing its mean over time (:321-329):

        loc' = loc + MLP(z_0) - loc.mean(axis=2)

    brightnessfc = MLP(latent_dim, 1, [model_dim]) (:284) on the HIP linear kernels;
    the gather of token 0 and the mean-removal shift are two small HIP kernels
    (vaesne_bright_input_*, vaesne_bright_shift_*).  Constructor signature of the
    reference (no `concat`: the encoder uses its default, concat=True)."""

    def __init__(self, num_bands=6, latent_len=8, latent_dim=4, model_dim=64, num_heads=4,
                 ff_dim=64, num_layers=4, dropout=0.1, selfattn=False, beta=1.,
                 prior=dist.Laplace, likelihood=dist.Laplace, posterior=dist.Laplace,
                 photometric_length=None):
        assert latent_len > 1, "first token for overall brightness"
        super().__init__(num_bands=num_bands, latent_len=latent_len, latent_dim=latent_dim,
                         model_dim=model_dim, num_heads=num_heads, ff_dim=ff_dim,
                         num_layers=num_layers, dropout=dropout, selfattn=selfattn, concat=True,
                         beta=beta, prior=prior, likelihood=likelihood, posterior=posterior)
        self.brightnessfc = MLP(latent_dim, 1, [model_dim])

    def decode_params(self, zs, x, groups=1, prepared=None):
        loc, scale = super().decode_params(zs, x, groups, prepared)
        brightness = self.brightnessfc(_ops.bright_input(zs))     # [K, groups*B, 1]
        return _ops.bright_shift(loc, brightness), scale
