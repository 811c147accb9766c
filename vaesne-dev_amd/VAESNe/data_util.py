"""Batch layout of the multimodal training data — reference data_util.py:10-20.

A batch is `[(flux, time, band, mask), (flux, wavelength, phase, mask)]`
(photometry, spectra), as produced by zipping two TensorDatasets.  The
reference's image datasets (data_util.py:23-79, torchvision/PIL) are outside
this build's scope.
"""
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
