"""Plotting helpers of the reference's evaluation scripts (plot_util.py:3-39;
used by cannon/test/goldstein/plot_masking.py).  Presentation only: matplotlib on
host arrays, nothing from the training step."""
import matplotlib.pyplot as plt
import numpy as np

LSST_BANDS = ("u", "g", "r", "i", "z", "y")
BAND_COLORS = ("purple", "blue", "darkgreen", "lime", "orange", "red")


def plot_lsst_lc(photoband, photomag, phototime, photomask, ax=None, label=False, s=5, lw=2):
    """Observed points of a 6-band light curve, one colour per band (scatter + a
    line through each band's points), magnitude axis inverted."""
    keep = ~photomask
    band, mag, time = photoband[keep], photomag[keep], phototime[keep]
    if ax is None:
        _, ax = plt.subplots()
    for b, (name, color) in enumerate(zip(LSST_BANDS, BAND_COLORS)):
        sel = np.where(band == b)[0]
        if len(sel) == 0:
            continue
        ax.scatter(time[sel], mag[sel], s=s, color=color, **({"label": name} if label else {}))
        ax.plot(time[sel], mag[sel], color=color, alpha=0.5, lw=lw)
    ax.invert_yaxis()
    # the reference returns nothing (its `return fig` sits under `if ax is None`
    # after ax was assigned, plot_util.py:20-21)


def plot_spectra_samples(spectra, wavelength, mask, alpha_level=0.1, ax=None, color="blue",
                         label=None):
    """Mean of spectrum samples [S, L] and its central (1 - alpha_level) band over the
    unmasked wavelengths."""
    if ax is None:
        _, ax = plt.subplots()
    keep = ~mask
    mean = np.nanmean(spectra, axis=0)
    lo = np.nanquantile(spectra, q=alpha_level / 2, axis=0)
    hi = np.nanquantile(spectra, q=1. - alpha_level / 2, axis=0)
    ax.plot(wavelength[keep], mean[keep], label=label, color=color)
    ax.fill_between(wavelength[keep], lo[keep], hi[keep], color=color, alpha=0.3)
