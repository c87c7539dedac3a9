"""1-D friends-of-friends clustering (riptide/clustering.py:4-50)."""
import numpy as np


def cluster1d(x, r, already_sorted=False):
    """Split points into clusters where consecutive sorted points are <= r apart.
    Returns a list of index arrays into x."""
    x = np.asarray(x)
    if not len(x):
        return []
    order = np.arange(len(x)) if already_sorted else x.argsort()
    gaps = np.abs(np.diff(x[order])) > r
    cuts = np.flatnonzero(gaps) + 1
    if not cuts.size:
        return [order]
    return np.split(order, cuts)
