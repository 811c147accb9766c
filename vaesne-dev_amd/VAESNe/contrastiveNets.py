"""Contrastive photometry/spectra pretraining network, MI355X build
(reference: contrastiveNets.py:20-101, ContraPhotSpec; trained with
losses.negInfoNCE by cannon/test_photospectra_contrast.py:96-127).

The two encoders are the VAE encoders' modules (HIP encoder blocks), the
projections are singlelayerMLPs on the HIP linear kernels, and the objective
is the fused InfoNCE kernel chain (losses.negInfoNCE).  Module attribute
names, constructor kwargs and state_dict keys follow the reference.
"""
import torch
from torch import nn

from .PhotometricLayers import photometricTransformerEncoder
from .SpectraLayers import spectraTransformerEncoder
from .util_layers import ReferencePickle, singlelayerMLP


class ContraPhotSpec(ReferencePickle, nn.Module):
    """contrastive photometric and spectra pretraining"""

    def __init__(self, latent_len, latent_dim, proj_dim,
                 num_bands, photo_model_dim, photo_num_heads, photo_ff_dim, photo_num_layers,
                 photo_dropout,
                 spec_model_dim, spec_num_heads, spec_num_layers, spec_ff_dim, spec_dropout,
                 selfattn):
        super().__init__()
        self.photometry_encoder = photometricTransformerEncoder(
            num_bands, latent_len, latent_dim, photo_model_dim, photo_num_heads, photo_ff_dim,
            photo_num_layers, photo_dropout, selfattn)
        self.photo_proj = singlelayerMLP(latent_len * latent_dim, proj_dim)
        self.spectra_encoder = spectraTransformerEncoder(
            latent_len, latent_dim, spec_model_dim, spec_num_heads, spec_num_layers,
            spec_ff_dim, spec_dropout, selfattn)
        self.spectra_proj = singlelayerMLP(latent_len * latent_dim, proj_dim)
        self.latent_dim = latent_dim
        self.latent_len = latent_len
        self.proj_dim = proj_dim

    def forward(self, x):
        photo_flux, time, band, photo_mask = x[0]
        spec_flux, wavelength, phase, spec_mask = x[1]
        z1 = self.photometry_encoder(photo_flux, time, band, photo_mask)
        # the reference passes (flux, wavelength, ...) into the encoder's
        # (wavelength, flux, ...) slots (contrastiveNets.py:79); kept as is
        z2 = self.spectra_encoder(spec_flux, wavelength, phase, spec_mask)
        z1 = self.photo_proj(z1.reshape(z1.shape[0], -1))
        z2 = self.spectra_proj(z2.reshape(z2.shape[0], -1))
        return z1, z2

    def photo_enc(self, x):
        photo_flux, time, band, photo_mask = x
        self.eval()
        with torch.no_grad():
            return self.photometry_encoder(photo_flux, time, band, photo_mask)

    def spectra_enc(self, x):
        self.eval()
        spec_flux, wavelength, phase, spec_mask = x
        with torch.no_grad():
            return self.spectra_encoder(spec_flux, wavelength, phase, spec_mask)
