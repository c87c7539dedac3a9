"""riptide_amd: MI355X-native FFA periodogram engine with riptide's Python API.

The compute path (downsampling ladder, FFA transform, boxcar S/N, running
median dereddening, normalisation) runs in hand-written HIP kernels for gfx950
behind the C ABI in include/riptide_amd.h; ``riptide_amd.libcpp`` is a drop-in
for riptide's ``riptide.libcpp`` module.
"""
__version__ = "0.1.0"

from .clustering import cluster1d
from .ffautils import generate_width_trials
from .metadata import Metadata
from .peak_detection import Peak, find_peaks
from .periodogram import Periodogram

# Compute API: needs the engine library (raises ImportError if it was not built)
from .libffa import boxcar_snr, downsample, ffa1, ffa2, ffafreq, ffaprd, generate_signal
from .running_medians import fast_running_median, running_median
from .search import ffa_search
from .time_series import TimeSeries

__all__ = [
    "TimeSeries", "Periodogram", "Metadata", "ffa_search", "ffa1", "ffa2", "ffafreq", "ffaprd",
    "generate_signal", "downsample", "boxcar_snr", "find_peaks", "running_median",
    "fast_running_median", "generate_width_trials", "cluster1d", "Peak",
]
