"""Batched peak detection of device-resident periodograms.

`find_peaks` of riptide (peak_detection.py:37-222) spends its time in two
data-parallel passes over the L x W S/N array of every trial: the per-segment
percentiles of segment_stats (np.percentile over every segment of every
width) and the dynamic-threshold mask poly(log f).  Both run here as HIP
kernels (rt_segment_order_stats_device, rt_threshold_select_device) on the
periodogram the engine left in HBM; only the order statistics (6 per
segment) and the selected row indices come back to the host.

The host finishes each stage with the reference's own numpy expressions:
numpy's 'linear' percentile (virtual index (n-1)q, _lerp with its t >= 0.5
branch) from the order statistics, np.polyfit / np.poly1d for the threshold
(batched bit for bit: polyfit_columns),
np.where order, cluster1d and the argmax per cluster -- so the peaks and
threshold polynomials are identical to riptide's for the same S/N.
"""
from math import ceil

import numpy as np

from . import _lib
from .clustering import cluster1d
from .peak_detection import Peak

_L = _lib.load()
_check = _lib.check

_QUANTILES = np.true_divide(np.array([25, 50, 75]), 100)     # np.percentile's q / 100


def _lerp(a, b, t):
    """numpy.lib._function_base_impl._lerp (numpy 2.x), elementwise."""
    diff_b_a = np.subtract(b, a)
    out = np.asanyarray(np.add(a, diff_b_a * t))
    np.subtract(b, diff_b_a * (1 - t), out=out, where=t >= 0.5, casting="unsafe", dtype=out.dtype)
    return out


def percentile_ranks(n):
    """Order-statistic ranks and interpolation weights numpy's 'linear'
    percentile uses for q = 25, 50, 75 on n sorted values."""
    vi = (n - 1) * _QUANTILES                        # _QuantileMethods['linear']
    prev = np.floor(vi)
    nxt = prev + 1
    above = vi >= n - 1                              # _get_indexes: both index -1 (the last value)
    prev[above] = -1
    nxt[above] = -1
    gamma = vi - prev                                # _get_gamma, before the -1 is resolved
    prev[above] = n - 1
    nxt[above] = n - 1
    ranks = np.stack([prev, nxt], axis=1).astype(np.uint32).ravel()     # [q25lo, q25hi, q50lo, ...]
    return ranks, gamma


def _lstsq_error(err, flag):
    raise np.linalg.LinAlgError("SVD did not converge in Linear Least Squares")


def polyfit_columns(x, Y, deg):
    """np.polyfit(x, Y[k], deg) for every row k of Y, bit for bit, in one
    call: polyfit's own steps (numpy/lib/_polynomial_impl.py: x + 0.0, the
    Vandermonde scaled by its column norms, rcond = len(x) eps, lstsq, the
    coefficients divided by the scale) with the lstsq gufunc looping over the
    rows as a batch -- one LAPACK gelsd per row with a single right-hand
    side, exactly polyfit's call (np.linalg.lstsq of a 1-D y), where a
    multi-column lstsq would round differently.  About 6 x faster than a
    Python loop of polyfit at cfg5's 16 x 13 fits per range."""
    from numpy.linalg import _umath_linalg
    x = np.asarray(x) + 0.0
    lhs = np.vander(x, int(deg) + 1)
    scale = np.sqrt((lhs * lhs).sum(axis=0))
    lhs /= scale
    rcond = len(x) * np.finfo(x.dtype).eps
    Y = np.asarray(Y) + 0.0
    with np.errstate(call=_lstsq_error, invalid="call", over="ignore", divide="ignore", under="ignore"):
        c = _umath_linalg.lstsq(lhs, Y[:, :, np.newaxis], rcond, signature="ddd->ddid")[0][..., 0]
    return c / scale


def poly1d_coefficients(c):
    """np.poly1d(c).coefficients: leading zeros trimmed, [0.] if none left."""
    c = np.trim_zeros(np.atleast_1d(c), trim="f")
    return c if c.size else np.array([0.0])


def poly1d_table(fits):
    """poly1d_coefficients of every fit in a [B, W, deg + 1] array at once:
    (the kernel's coefficient table -- leading zeros of either sign, as
    np.trim_zeros sees them, stored as +0, and 0 * x + c = c keeps
    np.polyval's value exactly -- and the reference's polyco of every
    (trial, width), [0.] for an all-zero fit)."""
    B, W, n = fits.shape
    lead = np.logical_and.accumulate(fits == 0, axis=-1)
    first = lead.sum(axis=-1)
    coeffs = np.where(lead, 0.0, fits)
    polycos = [[fits[b, iw, first[b, iw]:] if first[b, iw] < n else np.array([0.0])
                for iw in range(W)] for b in range(B)]
    return coeffs, polycos


def percentiles_from_order_stats(stats, gamma):
    """(s25, smed, s75) float64 arrays from the [..., 6] order statistics."""
    x = np.asarray(stats, dtype=np.float64)
    out = []
    for k in range(3):
        a, b = x[..., 2 * k], x[..., 2 * k + 1]
        out.append(_lerp(a, b, gamma[k]))
    return out


class PeakFinder:
    """find_peaks for every trial of a PeriodogramPlan's batched output.

    The plan's constants -- trial frequencies, log f, the segment layout and
    the segment centre frequencies (np.median of each segment) -- are computed
    once; `__call__` takes the device S/N [B, L, W] of `plan.run`.
    """

    def __init__(self, plan, tobs, smin=6.0, segwidth=5.0, nstd=6.0, minseg=10, polydeg=2, clrad=0.1,
                 max_selected=1 << 16):
        import torch
        self.plan = plan
        self.tobs = float(tobs)
        self.smin, self.segwidth, self.nstd = float(smin), float(segwidth), float(nstd)
        self.minseg, self.polydeg, self.clrad = int(minseg), int(polydeg), float(clrad)
        periods, foldbins = plan.grid()
        self.periods, self.foldbins = periods, foldbins
        self.freqs = 1.0 / periods                                  # Periodogram.freqs
        f = self.freqs
        L = f.size
        self.L, self.W = L, plan.num_widths
        # segment_stats (peak_detection.py:67-81)
        w = self.segwidth / self.tobs
        self.nseg = ceil(abs(f[-1] - f[0]) / w) if L else 0
        self.per_seg = L // self.nseg if self.nseg else 0
        n = self.nseg * self.per_seg
        self.device_ok = 0 < self.per_seg <= 32768      # kMaxSegmentPoints (peaks_kernels.hip)
        if self.device_ok:
            self.fc = np.median(f[:n].reshape(self.nseg, self.per_seg), axis=1)
            self.logfc = np.log(self.fc)
            self.ranks, self.gamma = percentile_ranks(self.per_seg)
        self.logf = torch.from_numpy(np.log(f)).to(plan.device)
        self.ncoef = self.polydeg + 1 if self.nseg >= self.minseg else 1
        self.cap = int(min(max_selected, max(L, 1)))

    def _threshold_polys(self, stats):
        """Per (trial, width) threshold coefficients and the reference's polyco."""
        s25, smed, s75 = percentiles_from_order_stats(stats, self.gamma)
        sstd = (s75 - s25) / 1.349
        sc = smed + self.nstd * sstd
        B, W = sc.shape[0], sc.shape[1]
        if len(self.fc) < self.minseg:
            coeffs = np.zeros((B, W, 1), dtype=np.float64)
            coeffs[..., 0] = poly1d_coefficients([self.smin])[-1]
            return coeffs, [[[self.smin] for _ in range(W)] for _ in range(B)]
        fits = polyfit_columns(self.logfc, sc.reshape(B * W, -1), self.polydeg).reshape(B, W, -1)
        return poly1d_table(fits)

    def __call__(self, snr, dms=None, stream=None):
        """Peaks of every trial: list of (peaks sorted by S/N, polycos).
        Kernels, allocations and copies all run on `stream` (default: the
        current stream)."""
        import torch
        s = stream if stream is not None else torch.cuda.current_stream(snr.device)
        with torch.cuda.stream(s):
            return self._run(snr, dms, s)

    def _run(self, snr, dms, stream):
        import torch
        from .engine import _stream_handle
        if snr.dim() == 2:
            snr = snr.unsqueeze(0)
        B, L, W = snr.shape
        if L != self.L or W != self.W or snr.dtype != torch.float32 or not snr.is_contiguous():
            raise ValueError("snr must be a contiguous float32 [B, L, W] tensor of the plan's shape")
        dms = list(dms) if dms is not None else [None] * B
        if not self.device_ok:
            return [self._host_trial(snr[b].cpu().numpy(), dms[b]) for b in range(B)]
        dev = snr.device
        sh = _stream_handle(stream)
        stats = torch.empty((B, W, self.nseg, 6), dtype=torch.float32, device=dev)
        ranks = np.ascontiguousarray(self.ranks, dtype=np.uint32)
        _check(_L.rt_segment_order_stats_device(_lib.ptr(snr), B, L * W, L, W, self.nseg, self.per_seg,
                                                _lib.ptr(ranks), ranks.size, _lib.ptr(stats), sh))
        coeffs, polycos = self._threshold_polys(stats.cpu().numpy())
        d_coeffs = torch.from_numpy(coeffs).to(dev)
        counts = torch.empty(B * W, dtype=torch.int32, device=dev)
        idx = torch.empty(B * W * self.cap, dtype=torch.int32, device=dev)
        _check(_L.rt_threshold_select_device(_lib.ptr(snr), B, L * W, L, W, _lib.ptr(self.logf), _lib.ptr(d_coeffs),
                                             coeffs.shape[2], self.smin, _lib.ptr(counts), _lib.ptr(idx), self.cap,
                                             sh))
        counts_h = counts.cpu().numpy().astype(np.int64)
        maxc = int(min(counts_h.max(initial=0), self.cap))
        lists = idx.view(B * W, self.cap)[:, :maxc].cpu().numpy().astype(np.int64) if maxc else None
        # selected rows of every (trial, width) in np.where order
        sel = {}
        host_cols = {}
        for b in range(B):
            for iw in range(W):
                c = int(counts_h[b * W + iw])
                if c > self.cap:          # truncated list: the column's mask on the host
                    col = snr[b, :, iw].double().cpu().numpy()
                    thr = np.poly1d(polycos[b][iw])(np.log(self.freqs))
                    sel[b, iw] = np.where((col > thr) & (col > self.smin))[0]
                    host_cols[b, iw] = col
                elif c:
                    sel[b, iw] = np.sort(lists[b * W + iw, :c])
        # S/N of every selected row, one gather
        keys = [k for k in sel if k not in host_cols and sel[k].size]
        svals = {}
        if keys:
            flat = np.concatenate([k[0] * L * W + sel[k] * W + k[1] for k in keys])
            got = torch.take(snr.reshape(-1), torch.from_numpy(flat).to(dev)).double().cpu().numpy()
            o = 0
            for k in keys:
                svals[k] = got[o:o + sel[k].size]
                o += sel[k].size
        for k, col in host_cols.items():
            svals[k] = col[sel[k]]
        results = []
        for b in range(B):
            peaks = []
            for iw in range(W):
                if (b, iw) not in svals or not sel[b, iw].size:
                    continue
                rows, s_sel = sel[b, iw], svals[b, iw]
                width = int(self.plan.widths[iw])
                # find_peaks_single / find_peaks (peak_detection.py:136-218)
                for cl in cluster1d(self.freqs[rows], self.clrad / self.tobs):
                    j = cl[s_sel[cl].argmax()]
                    ip = int(rows[j])
                    freq = float(self.freqs[ip])
                    peaks.append(Peak(period=float(1.0 / freq), freq=freq, width=width,
                                      ducy=float(float(width) / self.foldbins[ip]), iw=int(iw), ip=ip,
                                      snr=float(s_sel[j]), dm=dms[b]))
            peaks = sorted(peaks, key=lambda p: p.snr, reverse=True)
            results.append((peaks, {iw: polycos[b][iw] for iw in range(W)}))
        return results

    def _host_trial(self, snrs, dm):
        """The reference computation on the host (segments too long for the
        device sort, or degenerate layouts)."""
        from .peak_detection import find_peaks
        from .periodogram import Periodogram
        pg = Periodogram(self.plan.widths, self.periods, self.foldbins, snrs,
                         metadata={"dm": dm, "tobs": self.tobs})
        return find_peaks(pg, smin=self.smin, segwidth=self.segwidth, nstd=self.nstd, minseg=self.minseg,
                          polydeg=self.polydeg, clrad=self.clrad)
