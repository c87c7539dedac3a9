"""Boxcar width trials (riptide/ffautils.py:3-10)."""
import numpy as np


def generate_width_trials(nbins, ducy_max=0.20, wtsp=1.5):
    """Widths 1, then w <- max(w + 1, int(wtsp * w)) while w <= max(1, int(ducy_max * nbins))."""
    wmax = int(max(1, ducy_max * nbins))
    widths = []
    w = 1
    while w <= wmax:
        widths.append(w)
        w = int(max(w + 1, wtsp * w))
    return np.asarray(widths)
