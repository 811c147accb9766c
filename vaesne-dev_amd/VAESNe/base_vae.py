"""VAE base class — base_vae.py:9-35 of the reference (attribute contract:
pz / px_z / qz_x distribution classes, enc, dec, llik_scaling, pz_params)."""
import torch
import torch.nn as nn


class VAE(nn.Module):
    def __init__(self, prior_dist, likelihood_dist, post_dist, enc, dec, params):
        super().__init__()
        self.pz = prior_dist
        self.px_z = likelihood_dist
        self.qz_x = post_dist
        self.enc = enc
        self.dec = dec
        self.modelName = None
        self.params = params
        self._pz_params = None  # defined in subclass
        self._qz_x_params = None  # populated in `forward`
        self.llik_scaling = 1.0

    @property
    def pz_params(self):
        return self._pz_params

    @property
    def qz_x_params(self):
        if self._qz_x_params is None:
            raise NameError("qz_x params not initalised yet!")
        return self._qz_x_params

    @staticmethod
    def getDataLoaders(batch_size, shuffle=True, device="cuda"):
        raise NotImplementedError

    # distribution construction without argument validation: validation would
    # synchronise the device (and break hipGraph capture); the kernels produce
    # finite loc and positive scale by construction.
    def _dist(self, cls, loc, scale):
        return cls(loc, scale, validate_args=False)


def check_laplace(*classes):
    import torch.distributions as dist
    for c in classes:
        if c is not dist.Laplace:
            raise NotImplementedError(
                "the MI355X VAESNe build implements the reference's Laplace prior/likelihood/"
                f"posterior (SURVEY.md F1); got {c}")
