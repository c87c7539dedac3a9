"""Dynamic-threshold peak finding in a periodogram (riptide/peak_detection.py:14-222).

Host-side (numpy) stage that consumes the S/N the engine produces; SURVEY.md
§8(f1) ranks moving it to the GPU next.  The computation is the reference's,
expression for expression, so candidate lists are identical for identical S/N.
"""
import logging
import typing
from math import ceil

import numpy as np

from .clustering import cluster1d
from .timing import timing

log = logging.getLogger("riptide.peak_detection")


class Peak(typing.NamedTuple):
    """A periodogram peak (peak_detection.py:14-34)."""
    period: float
    freq: float
    width: int
    ducy: float
    iw: int
    ip: int
    snr: float
    dm: float

    def summary_dict(self):
        return {a: getattr(self, a) for a in ("period", "freq", "dm", "width", "ducy", "snr")}


def segment_stats(f, s, T, segwidth=5.0):
    """Centre frequency, median S/N and IQR-based S/N sigma of consecutive
    frequency segments of width segwidth / T (peak_detection.py:37-84)."""
    nseg = ceil(abs(f[-1] - f[0]) / (segwidth / T))
    per_seg = len(f) // nseg
    used = nseg * per_seg
    fseg = f[:used].reshape(nseg, per_seg)
    sseg = s[:used].reshape(nseg, per_seg)
    fc = np.median(fseg, axis=1)
    q25, q50, q75 = np.percentile(sseg, (25, 50, 75), axis=-1)
    return fc, q50, (q75 - q25) / 1.349


def fit_threshold(fc, tc, polydeg=2):
    """Polynomial in log(f) through the control points (peak_detection.py:87-108)."""
    return np.poly1d(np.polyfit(np.log(fc), tc, polydeg))


def find_peaks_single(f, s, T, smin=6.0, segwidth=5.0, nstd=7.0, minseg=10, polydeg=2, clrad=0.1):
    """Peak centre indices for one width trial, and the threshold polynomial
    coefficients (peak_detection.py:111-142)."""
    fc, smed, sstd = segment_stats(f, s, T, segwidth=segwidth)
    if len(fc) >= minseg:
        poly = fit_threshold(fc, smed + nstd * sstd, polydeg=polydeg)
        polyco = poly.coefficients
    else:
        polyco = [smin]
        poly = np.poly1d(polyco)
    selected = np.where((s > poly(np.log(f))) & (s > smin))[0]
    centres = []
    for members in cluster1d(f[selected], clrad / T):
        idx = selected[members]
        centres.append(idx[s[idx].argmax()])
    return centres, polyco


@timing
def find_peaks(pgram, smin=6.0, segwidth=5.0, nstd=6.0, minseg=10, polydeg=2, clrad=0.1):
    """Significant peaks of a Periodogram, sorted by decreasing S/N, and the
    per-width threshold polynomials {iw: coefficients} (peak_detection.py:145-222)."""
    f = pgram.freqs
    T = pgram.tobs
    dm = pgram.metadata["dm"]
    peaks, polycos = [], {}
    for iw, width in enumerate(pgram.widths):
        s = pgram.snrs[:, iw].astype(float)
        centres, polycos[iw] = find_peaks_single(
            f, s, T, smin=smin, segwidth=segwidth, nstd=nstd, minseg=minseg, polydeg=polydeg, clrad=clrad)
        for ip in centres:
            peaks.append(Peak(
                period=float(1.0 / f[ip]), freq=float(f[ip]), width=int(width),
                ducy=float(float(width) / pgram.foldbins[ip]), iw=int(iw), ip=int(ip),
                snr=float(s[ip]), dm=dm))
    peaks.sort(key=lambda p: p.snr, reverse=True)
    return peaks, polycos
