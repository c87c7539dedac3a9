"""Running medians (riptide/running_medians.py:5-83), computed on the GPU."""
import numpy as np

from . import libcpp


def running_median(x, width_samples):
    """Exact running median, odd window < len(x), edges replicated (running_medians.py:5-37)."""
    return libcpp.running_median(np.ascontiguousarray(x), width_samples)


def scrunch(data, factor):
    """Mean of consecutive blocks of `factor` samples, tail dropped (running_medians.py:40-46)."""
    factor = int(factor)
    n = (data.size // factor) * factor
    return data[:n].reshape(-1, factor).mean(axis=1)


def fast_running_median(data, width_samples, min_points=101):
    """Running median of a scrunched copy (>= min_points samples per window),
    linearly interpolated back to full resolution (running_medians.py:49-83).
    float64 output, float32 when no scrunching is needed (as the reference)."""
    if not (min_points % 2):
        raise ValueError("min_points must be an odd number")
    factor = int(max(1, width_samples / float(min_points)))
    if factor == 1:
        return running_median(data, width_samples)
    data = np.asarray(data)
    if data.dtype != np.float32:
        # non-float32 input: the reference scrunches in the input dtype before
        # the (float32) running median; keep that order
        lores = scrunch(data, factor)
        rmed = running_median(lores, min_points)
        x_lores = np.arange(lores.size) * factor + 0.5 * (factor - 1)
        return np.interp(np.arange(data.size), x_lores, rmed)
    return libcpp.fast_running_median_scrunched(data, width_samples, min_points)
