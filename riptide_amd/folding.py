"""Candidate folding (riptide/folding.py:1-81) with the
engine's real-factor downsampling: the series is downsampled by
period / bins / tsamp on the GPU (rt_downsample), cut into whole periods and
scaled exactly as the reference does (numpy, float32); the vertical
downsampling to sub-integrations runs all phase-bin columns in one batched
GPU call (rt_downsample_rows) instead of one call per column.
"""
import numpy as np

from . import _lib
from .libffa import downsample


def downsample_rows(X, factor):
    """Downsample every row of a 2D float32 array by `factor` (one device call)."""
    X = np.ascontiguousarray(X, dtype=np.float32)
    rows, n = X.shape
    f = float(factor)
    if not ((f > 1.0) and (f <= n)):
        raise ValueError("Downsampling factor must verify: 1 < f <= size")
    L = _lib.load()
    out = np.empty((rows, int(L.rt_downsampled_size(n, f))), dtype=np.float32)
    if rows:
        _lib.check(L.rt_downsample_rows(_lib.ptr(X), rows, n, f, _lib.ptr(out)))
    return out


def downsample_vertical(X, factor):
    """Downsample a 2D array along its first axis (folding.py:6-16)."""
    m, _ = X.shape
    if not factor > 1:
        raise ValueError("factor must be > 1")
    if not factor < m:
        raise ValueError("factor must be strictly smaller than the number of input lines")
    return np.ascontiguousarray(downsample_rows(np.ascontiguousarray(X.T), factor).T)


def fold(ts, period, bins, subints=None):
    """Fold a TimeSeries at `period` seconds with `bins` phase bins
    (folding.py:19-81): a (subints, bins) array, or (bins,) when the result
    has a single sub-integration."""
    if period > ts.length:
        raise ValueError("Period exceeds data length")
    tbin = period / bins
    if not tbin > ts.tsamp:
        raise ValueError("Bin width is shorter than sampling time")
    if subints is not None:
        subints = int(subints)
        if not subints >= 1:
            raise ValueError("subints must be >= 1 or None")
        full_periods = ts.length / period
        if subints > full_periods:
            raise ValueError(f"subints ({subints}) exceeds the number of signal periods that fit in the data "
                             f"({full_periods})")
    factor = tbin / ts.tsamp
    data = downsample(ts.data, factor)
    m = data.size // bins
    folded = data[:m * bins].reshape(m, bins)
    folded *= (m * factor) ** -0.5
    if subints == 1 or m == 1:
        return folded.sum(axis=0)
    if subints is None or subints == m:
        return folded
    return downsample_vertical(folded, m / subints)
