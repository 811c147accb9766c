"""Downstream regression head on a frozen VAE encoder, MI355X build
(reference: regression.py:9-26, VAEregressionHead; driven by
cannon/photometry2goldstein_mmvae.py:55 and spec2goldstein_mmvae.py:56).

The encoder runs through the HIP kernels under `vae.encode` (eval mode, no
grad, posterior mean), the MLP head through the HIP linear kernels.  The
contrastive heads of the reference file (ContraPhotSpec consumers) are out of
scope.
"""
from torch import nn

from .util_layers import MLP


class VAEregressionHead(nn.Module):
    def __init__(self, vae, outdim, freeze_vae=True, MLPlatent=[64, 64]):
        super(VAEregressionHead, self).__init__()
        if freeze_vae:
            for param in vae.parameters():
                param.requires_grad = False
        self.vae = vae
        self.outfc = MLP(self.vae.latent_len * self.vae.latent_dim, outdim, MLPlatent)

    def forward(self, x):
        h = self.vae.encode(x, True)
        h = h.reshape(h.shape[0], -1)   # flatten the latent
        return self.outfc(h)
