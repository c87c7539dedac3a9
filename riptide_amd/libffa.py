"""Kernel-level API (riptide/libffa.py:15-243), backed by the HIP engine."""
import numpy as np
from numpy import cos, exp, log, pi, sin

from . import libcpp
from .ffautils import generate_width_trials  # noqa: F401  (re-export, as the reference module)


def generate_signal(nsamp, period, phi0=0.5, ducy=0.02, amplitude=10.0, stdnoise=1.0):
    """Von Mises pulse train of unit L2 norm times `amplitude`, plus Gaussian
    noise from numpy's global RNG (libffa.py:15-68).  Test-input generator."""
    kappa = log(2.0) / (2.0 * sin(pi * ducy / 2.0) ** 2)
    phase = (np.arange(nsamp, dtype=float) / period - phi0) * (2 * pi)
    signal = exp(kappa * (cos(phase) - 1.0))
    signal *= amplitude * (signal ** 2).sum() ** -0.5
    noise = np.random.normal(size=nsamp, loc=0.0, scale=stdnoise) if stdnoise > 0.0 else 0.0
    return signal + noise


def ffa2(data):
    """FFA transform of a 2D (m periods, p phase bins) array -> float32 (m, p)."""
    return libcpp.ffa2(data)


def ffa1(data, p):
    """FFA transform of a time series at base period p samples; the last
    N mod p samples are ignored (libffa.py:94-126)."""
    if not data.ndim == 1:
        raise ValueError("input data must be one-dimensional")
    if not (isinstance(p, int) and p > 0):
        raise ValueError("p must be an integer > 1")
    if p > data.size:
        raise ValueError("p must be smaller than the total number of samples")
    m = data.size // p
    return ffa2(data[:m * p].reshape(m, p))


def ffafreq(N, p, dt=1.0):
    """Trial frequencies of the FFA output rows (libffa.py:129-169):
    f_s = (1/p - s/(m-1) / p^2) / dt, s = 0..m-1, m = N // p."""
    if not (isinstance(N, int) and N > 0):
        raise ValueError("N must be a strictly positive integer")
    if not (isinstance(p, int) and p > 1):
        raise ValueError("p must be an integer > 1")
    if not N >= p:
        raise ValueError("p must be smaller than (or equal to) N")
    if not dt > 0:
        raise ValueError("dt must be strictly positive")
    f0 = 1.0 / p
    m = N // p
    if m == 1:
        f = np.asarray([f0])
    else:
        s = np.arange(m)
        f = f0 - s / (m - 1.0) * f0 ** 2
    return f / dt


def ffaprd(N, p, dt=1.0):
    """Trial periods of the FFA output rows (libffa.py:172-191)."""
    return 1.0 / ffafreq(N, p, dt=dt)


def boxcar_snr(data, widths, stdnoise=1.0):
    """Boxcar matched-filter S/N of profiles along the last axis, for each
    width; output shape data.shape[:-1] + (len(widths),) (libffa.py:194-225)."""
    widths = np.asarray(widths, dtype=np.uint64)
    b = data.shape[-1]
    snr = libcpp.snr2(data.reshape(-1, b).astype(np.float32), widths, stdnoise)
    return snr.reshape(list(data.shape[:-1]) + [widths.size])


def downsample(data, factor):
    """Downsample by a real-valued factor (libffa.py:228-243)."""
    return libcpp.downsample(data, factor)
