"""Drop-in replacement for riptide's native module ``riptide.libcpp``.

Same function names, argument names/defaults, output dtypes/shapes and
ValueError messages as the pybind11 module
(/root/reference/riptide/cpp/python_bindings.cpp:213-267), but every call runs
HIP kernels on the MI355X through the C ABI in include/riptide_amd.h.

Argument coercion mirrors pybind11's ``py::array_t<T>`` (forcecast): any
array-like is converted to float32 (widths to uint64); an input that is
already float32 but not C-contiguous is rejected exactly like the reference's
``assert_c_contiguous`` (python_bindings.cpp:21-29).
"""
import ctypes

import numpy as np

from . import _lib

_L = _lib.load()
_ptr = _lib.ptr
_check = _lib.check


def _as_f32(a, ndim):
    arr = np.asarray(a, dtype=np.float32)
    if not arr.flags.c_contiguous:
        raise ValueError("Input numpy array must be contiguous in memory")
    if arr.ndim != ndim:
        raise ValueError(f"array has incorrect number of dimensions: {arr.ndim}; expected {ndim}")
    return arr


def _as_widths(w):
    arr = np.asarray(w, dtype=np.uint64)
    if not arr.flags.c_contiguous:
        raise ValueError("Input numpy array must be contiguous in memory")
    if arr.ndim != 1:
        raise ValueError(f"array has incorrect number of dimensions: {arr.ndim}; expected 1")
    return arr


def _size_t(v, name):
    if isinstance(v, (bool, np.bool_)) or not isinstance(v, (int, np.integer)) or v < 0:
        raise TypeError(f"{name} must be a non-negative integer")
    return int(v)


def rollback(x, shift):
    """python_bindings.cpp:32-40: roll(x, -shift)."""
    x = _as_f32(x, 1)
    shift = _size_t(shift, "shift")
    out = np.empty(x.size, dtype=np.float32)
    _check(_L.rt_rollback(_ptr(x), x.size, shift, _ptr(out)))
    return out


def fused_rollback_add(x, y, shift):
    """python_bindings.cpp:43-58: x + roll(y, -shift)."""
    xa = np.asarray(x, dtype=np.float32)
    ya = np.asarray(y, dtype=np.float32)
    if xa.size != ya.size:
        raise ValueError("Arrays must have the same number of elements")
    xa = _as_f32(xa, 1)
    ya = _as_f32(ya, 1)
    shift = _size_t(shift, "shift")
    out = np.empty(xa.size, dtype=np.float32)
    _check(_L.rt_fused_rollback_add(_ptr(xa), _ptr(ya), xa.size, shift, _ptr(out)))
    return out


def circular_prefix_sum(x, nsum):
    """python_bindings.cpp:61-69."""
    x = _as_f32(x, 1)
    nsum = _size_t(nsum, "nsum")
    out = np.empty(nsum, dtype=np.float32)
    _check(_L.rt_circular_prefix_sum(_ptr(x), x.size, nsum, _ptr(out)))
    return out


def ffa2(data):
    """python_bindings.cpp:72-84: FFA transform of a 2D (rows, cols) array."""
    x = _as_f32(data, 2)
    rows, cols = x.shape
    out = np.empty((rows, cols), dtype=np.float32)
    _check(_L.rt_ffa2(_ptr(x), rows, cols, _ptr(out)))
    return out


def benchmark_ffa2(rows, cols, loops):
    """python_bindings.cpp:87-106: seconds per FFA transform of a rows x cols block."""
    sec = ctypes.c_double(0.0)
    _check(_L.rt_benchmark_ffa2(_size_t(rows, "rows"), _size_t(cols, "cols"), _size_t(loops, "loops"),
                                ctypes.byref(sec)))
    return sec.value


def snr1(data, widths, stdnoise=1.0):
    """python_bindings.cpp:109-126."""
    x = _as_f32(data, 1)
    w = _as_widths(widths)
    out = np.empty(w.size, dtype=np.float32)
    _check(_L.rt_snr1(_ptr(x), x.size, _ptr(w), w.size, float(stdnoise), _ptr(out)))
    return out


def snr2(data, widths, stdnoise=1.0):
    """python_bindings.cpp:129-148."""
    x = _as_f32(data, 2)
    w = _as_widths(widths)
    rows, cols = x.shape
    out = np.empty((rows, w.size), dtype=np.float32)
    _check(_L.rt_snr2(_ptr(x), rows, cols, _ptr(w), w.size, float(stdnoise), _ptr(out)))
    return out


def downsample(data, factor):
    """python_bindings.cpp:151-165: real-factor downsampling."""
    x = _as_f32(data, 1)
    f = float(factor)
    if not ((f > 1.0) and (f <= x.size)):
        raise ValueError("Downsampling factor must verify: 1 < f <= size")
    out = np.empty(int(_L.rt_downsampled_size(x.size, f)), dtype=np.float32)
    _check(_L.rt_downsample(_ptr(x), x.size, f, _ptr(out)))
    return out


def periodogram(data, tsamp, widths, period_min, period_max, bins_min, bins_max):
    """python_bindings.cpp:168-197: (periods f64[L], foldbins u32[L], snrs f32[L, W])."""
    x = _as_f32(data, 1)
    w = _as_widths(widths)
    bmin, bmax = _size_t(bins_min, "bins_min"), _size_t(bins_max, "bins_max")
    length = ctypes.c_size_t(0)
    _check(_L.rt_periodogram_length(x.size, float(tsamp), float(period_min), float(period_max), bmin, bmax,
                                    ctypes.byref(length)))
    L = length.value
    periods = np.empty(L, dtype=np.float64)
    foldbins = np.empty(L, dtype=np.uint32)
    snrs = np.empty((L, w.size), dtype=np.float32)
    _check(_L.rt_periodogram(_ptr(x), x.size, float(tsamp), _ptr(w), w.size, float(period_min),
                             float(period_max), bmin, bmax, _ptr(periods), _ptr(foldbins), _ptr(snrs)))
    return periods, foldbins, snrs


def running_median(data, width):
    """python_bindings.cpp:200-210: exact running median, odd width < size."""
    x = _as_f32(data, 1)
    width = _size_t(width, "width")
    out = np.empty(x.size, dtype=np.float32)
    _check(_L.rt_running_median(_ptr(x), x.size, width, _ptr(out)))
    return out


# ---- engine extensions used by the Python layer (not in the reference module)
def fast_running_median_scrunched(data, width_samples, min_points):
    x = _as_f32(data, 1)
    out = np.empty(x.size, dtype=np.float64)
    _check(_L.rt_fast_running_median(_ptr(x), x.size, int(width_samples), int(min_points), _ptr(out)))
    return out


def deredden_normalise(data, width_samples, min_points, deredden=True, normalise=True):
    x = _as_f32(data, 1)
    out = np.empty(x.size, dtype=np.float32)
    _check(_L.rt_deredden_normalise(_ptr(x), x.size, int(width_samples), int(min_points), int(bool(deredden)),
                                    int(bool(normalise)), _ptr(out)))
    return out
