"""Spectra VAE, MI355X build (reference: SpectraVAE.py:11-332).

Constructors accept and ignore `spectra_length` (the cannon scripts pass it,
SURVEY.md F9).
"""
import torch
import torch.distributions as dist
from torch import nn

from . import _chain, _ops
from .SpectraLayers import spectraTransformerDecoder, spectraTransformerEncoder
from .base_vae import VAE, check_laplace
from .util_layers import MLP, ReferencePickle


class SpectraEnc(nn.Module):
    """SpectraVAE.py:11-51."""

    def __init__(self, latent_len, latent_dim, model_dim, num_heads, num_layers, ff_dim,
                 dropout=0.1, selfattn=False, concat=True):
        super().__init__()
        self.inference_transformer = spectraTransformerEncoder(
            2 * latent_len, latent_dim, model_dim, num_heads, num_layers, ff_dim, dropout,
            selfattn, concat)
        self.latent_dim = latent_dim
        self.latent_len = latent_len

    def forward(self, flux, wavelength, phase, mask=None):
        return _chain.drive([self.steps(flux, wavelength, phase, mask)])[0]

    def steps(self, flux, wavelength, phase, mask=None):
        # NB argument order into the encoder is the reference's (see SpectraLayers)
        bottleneck = yield from self.inference_transformer.steps(flux, wavelength, phase, mask)
        return _ops.latent_head(bottleneck, self.latent_len)


class SpectraDec(nn.Module):
    """SpectraVAE.py:53-87: returns (loc, 1 + 1e10*mask)."""

    def __init__(self, latent_dim, model_dim, num_heads, ff_dim, num_layers, dropout=0.1,
                 selfattn=False):
        super().__init__()
        self.generativetransformer = spectraTransformerDecoder(
            latent_dim, model_dim, num_heads, ff_dim, num_layers, dropout, selfattn)

    def pxz(self, wavelength, phase, z, mask=None, repeat=1, prepared=None):
        return self.generativetransformer(wavelength, phase, z, mask, repeat=repeat, prepared=prepared)

    def forward(self, wavelength, phase, z, mask=None, repeat=1, prepared=None):
        x_rec = self.pxz(wavelength, phase, z, mask, repeat=repeat, prepared=prepared)
        if mask is None:
            var = torch.ones_like(x_rec)
        else:
            var = _ops.mask_scale(mask, 1, 1e10, x_rec).view_as(x_rec)
        return x_rec, var


class SpectraVAE(ReferencePickle, VAE):
    def __init__(self, latent_len=4, latent_dim=2, model_dim=32, num_heads=4, ff_dim=32,
                 num_layers=4, dropout=0.1, selfattn=False, concat=True, beta=1.,
                 prior=dist.Laplace, likelihood=dist.Laplace, posterior=dist.Laplace,
                 spectra_length=None):
        check_laplace(prior, likelihood, posterior)
        super().__init__(
            prior, likelihood, posterior,
            SpectraEnc(latent_len, latent_dim, model_dim, num_heads, num_layers, ff_dim,
                       dropout, selfattn, concat),
            SpectraDec(latent_dim, model_dim, num_heads, ff_dim, num_layers, dropout),
            params=[latent_len, latent_dim, model_dim, num_heads, num_layers, ff_dim, dropout,
                    selfattn])
        self._pz_params = nn.ParameterList([
            nn.Parameter(torch.zeros(latent_len, latent_dim), requires_grad=False),
            nn.Parameter(torch.ones(latent_len, latent_dim), requires_grad=False),
        ])
        self.llik_scaling = 1. / beta
        self.modelName = 'spectrum'
        self.latent_len = latent_len
        self.latent_dim = latent_dim

    def forward(self, x, K=1):
        """SpectraVAE.py:148-165 -> (qz_x, px_z, zs)."""
        qz_x, zs = self.posterior(x, K)
        px_z = self.decode(zs, x)
        return qz_x, px_z, zs

    def posterior(self, x, K=1):
        """Encoder -> q(z|x) and K reparameterised draws (SpectraVAE.py:149-152)."""
        return _chain.drive([self.posterior_steps(x, K)])[0]

    def posterior_steps(self, x, K=1):
        """posterior as a generator (VAESNe._chain.drive)."""
        params = yield from self.encoder_steps(x)
        return self.sample(params, K)

    def encoder_steps(self, x):
        """The encoder alone as a generator (-> (loc, scale) of q(z|x))."""
        flux, wavelength, phase, mask = x
        return (yield from self.enc.steps(flux, wavelength, phase, mask))

    def sample(self, params, K=1):
        """q(z|x) of the encoder output `params` and its K reparameterised draws."""
        # q(z|x) reads aliases of (loc, scale) whose gradients the sampler's backward adds
        z, *params = _ops.posterior_rsample(*params, K)
        self._qz_x_params = tuple(params)
        return self._dist(self.qz_x, *params), z

    def reconstruct(self, x, K=1):
        self.eval()
        with torch.no_grad():
            mu, scale = self.enc(*x)
            zs = _ops.laplace_rsample(mu, scale, K)
            return self.decode(zs, x).mean

    def encode(self, x, mean=True):
        flux, wavelength, phase, mask = x
        self.eval()
        with torch.no_grad():
            qz_x = self._dist(self.qz_x, *self.enc(flux, wavelength, phase, mask))
        if mean:
            return qz_x.mean
        return qz_x

    def decode(self, zs, x):
        """SpectraVAE.py:186-196."""
        return self._dist(self.px_z, *self.decode_params(zs, x))

    def _dec_inputs(self, x, K, groups):
        _, wavelength, phase, mask = x
        B, L = wavelength.shape
        rep = lambda t: t.unsqueeze(0).unsqueeze(0).expand(K, groups, B, L).reshape(-1, L)
        return (wavelength, phase.unsqueeze(0).unsqueeze(0).expand(K, groups, B).reshape(-1),
                None if mask is None else rep(mask))

    def decode_prepare(self, x, K, groups=1):
        """The latent-independent part of decode_params(zs, x, groups) for K samples
        (embeddings, block 1's in-projection and self-attention):
        -> `prepared` for decode_params."""
        wavelength, phase, mask = self._dec_inputs(x, K, groups)
        return (K, groups, mask, self.dec.generativetransformer.prepare(
            wavelength, phase, mask, repeat=K * groups, lc=self.latent_len + 1))

    def decode_params(self, zs, x, groups=1, prepared=None):
        """(loc, scale) [K, groups*B, L] for latents zs [K, groups*B, Lz, Dz]
        decoded at x's grid, x's batch repeated `groups` times (group-major).
        `prepared`: decode_prepare(x, K, groups) computed ahead."""
        K = zs.shape[0]
        B, L = x[1].shape
        if prepared is not None and prepared[:2] == (K, groups):
            wavelength, phase = x[1], None
            mask, pre = prepared[2], prepared[3]
        else:
            (wavelength, phase, mask), pre = self._dec_inputs(x, K, groups), None
        # the wavelength embedding runs once per distinct spectrum (repeat = K * groups)
        loc, scale = self.dec(wavelength, phase, zs.reshape(-1, zs.shape[-2], zs.shape[-1]), mask,
                              repeat=K * groups, prepared=pre)
        return loc.reshape(K, groups * B, L), scale.reshape(K, groups * B, L)

    def generate(self, N, x):
        """SpectraVAE.py:198-206: N prior draws decoded at x's grids."""
        self.eval()
        with torch.no_grad():
            loc, scale = self.pz_params[0], self.pz_params[1]
            zs = _ops.laplace_rsample(loc.unsqueeze(0).contiguous(), scale.unsqueeze(0).contiguous(), N)
            return self.decode(zs, x).mean.unsqueeze(0)


class BrightSpectraVAE(SpectraVAE):
    """SpectraVAE.py:211-332: the first latent token (with the phase) carries the
    spectrum's overall brightness.  decode() (:308-322):

        loc' = loc + MLP([z_0 | phase]) - loc.mean(axis=2)

    brightnessfc = MLP(latent_dim + 1, 1, [model_dim]) (:268).  Constructor signature
    of the reference (no `concat`: the encoder uses its default, concat=True)."""

    def __init__(self, latent_len=4, latent_dim=2, model_dim=32, num_heads=4, ff_dim=32,
                 num_layers=4, dropout=0.1, selfattn=False, beta=1., prior=dist.Laplace,
                 likelihood=dist.Laplace, posterior=dist.Laplace, spectra_length=None):
        assert latent_len > 1, "Need at least one token for overall brightness"
        super().__init__(latent_len=latent_len, latent_dim=latent_dim, model_dim=model_dim,
                         num_heads=num_heads, ff_dim=ff_dim, num_layers=num_layers,
                         dropout=dropout, selfattn=selfattn, concat=True, beta=beta, prior=prior,
                         likelihood=likelihood, posterior=posterior)
        self.brightnessfc = MLP(latent_dim + 1, 1, [model_dim])

    def decode_params(self, zs, x, groups=1, prepared=None):
        loc, scale = super().decode_params(zs, x, groups, prepared)
        phase = x[2]
        brightness = self.brightnessfc(_ops.bright_input(zs, phase))   # [K, groups*B, 1]
        return _ops.bright_shift(loc, brightness), scale
