"""Datasets and small data helpers — reference data_util.py.

  multimodalDataset       data_util.py:10-20  the batch layout of the multimodal step:
                          `[(flux, time, band, mask), (flux, wavelength, phase, mask)]`
                          (photometry, spectra), as produced by zipping two TensorDatasets
  ImagePathDataset        data_util.py:23-44  host-galaxy image files -> (image, empty label)
  ImagePathDatasetAug     data_util.py:47-73  the same with random flips / affine, `factor`x
  get_goldstein_params    data_util.py:76-79  the simulation parameters encoded in a file name

The reference imports torchvision and PIL at module top (data_util.py:3-5), which made
the whole module unimportable without torchvision.  Here they are
imported only when an image dataset needs them, so the training-step imports
(`multimodalDataset`, `get_goldstein_params`) work on any host.
"""
import re

import numpy as np
import torch
from torch.utils.data import Dataset


class multimodalDataset(Dataset):
    def __init__(self, *datasets):
        assert all(len(d) == len(datasets[0]) for d in datasets), "All datasets must be the same length"
        self.datasets = datasets
        self.num_modes = len(datasets)

    def __len__(self):
        return len(self.datasets[0])

    def __getitem__(self, idx):
        return tuple(d[idx] for d in self.datasets)


def _transforms():
    try:
        from torchvision import transforms
    except ImportError as e:   # the reference needs it too (data_util.py:5)
        raise ImportError("VAESNe image datasets need torchvision for their default transform "
                          "(pass transform=... to avoid it)") from e
    return transforms


def _default_transform(augment):
    """data_util.py:31-34 (plain) and :56-62 (augmented): to tensor, normalise every
    channel with mean 0.5 / std 0.5; the augmented one first flips both ways and
    applies a random affine (15 deg, 5 % shift, 0.75-1.25 scale)."""
    T = _transforms()
    head = [T.RandomHorizontalFlip(), T.RandomVerticalFlip(),
            T.RandomAffine(degrees=15, translate=(0.05, 0.05), scale=(0.75, 1.25))] if augment else []
    return T.Compose(head + [T.ToTensor(), T.Normalize(mean=[0.5, 0.5, 0.5], std=[0.5, 0.5, 0.5])])


class ImagePathDataset(Dataset):
    """Images read from `image_paths` as RGB; item = (transform(image), empty label)."""

    def __init__(self, image_paths, transform=None):
        self.image_paths = image_paths
        self.transform = transform or _default_transform(augment=False)

    def __len__(self):
        return len(self.image_paths)

    def _load(self, idx):
        from PIL import Image
        image = Image.open(self.image_paths[idx]).convert('RGB')
        if self.transform:
            image = self.transform(image)
        return image, torch.tensor([])

    def __getitem__(self, idx):
        return self._load(idx)


class ImagePathDatasetAug(ImagePathDataset):
    """Each image `factor` times (index wraps around), default transform augmented."""

    def __init__(self, image_paths, transform=None, factor=10):
        self.factor = factor
        self.image_paths = image_paths
        self.transform = transform or _default_transform(augment=True)

    def __len__(self):
        return len(self.image_paths) * self.factor

    def __getitem__(self, idx):
        return self._load(idx % len(self.image_paths))


_SCI = re.compile(r'[-+]?\d*\.\d+e[-+]?\d+')


def get_goldstein_params(filename):
    """Every scientific-notation number (`1.5e+00`, `-.3e-02`, ...) in `filename`, in
    order, as a float64 array (the goldstein simulation parameters the regression
    scripts use as targets, e.g. cannon/photometry2goldstein_mmvae.py)."""
    return np.array([float(v) for v in _SCI.findall(filename)])
