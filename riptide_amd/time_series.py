"""TimeSeries container (riptide/time_series.py:16-397).

Dereddening and normalisation run as HIP kernels (rt_deredden_normalise).
SIGPROC / PRESTO loaders: riptide_amd.reading.
"""
import copy as _copy

import numpy as np

from . import libcpp
from .libffa import downsample, generate_signal
from .metadata import Metadata
from .timing import timing


class TimeSeries:
    """Time series to be searched with the FFA.  Use the classmethods to create one."""

    def __init__(self, data, tsamp, metadata=None, copy=False):
        arr = np.asarray(data, dtype=np.float32)
        self._data = arr.copy() if copy else arr
        self._tsamp = float(tsamp)
        self.metadata = Metadata(metadata) if metadata is not None else Metadata({})
        self.metadata["tobs"] = self.length

    @property
    def data(self):
        return self._data

    @property
    def tsamp(self):
        return self._tsamp

    def copy(self):
        return _copy.deepcopy(self)

    def normalise(self, inplace=False):
        """Zero mean, unit variance (float64 statistics; time_series.py:66-90)."""
        out = libcpp.deredden_normalise(self.data, 0, 1, deredden=False, normalise=True)
        if inplace:
            self._data = out
        else:
            return TimeSeries(out, self.tsamp, metadata=self.metadata)

    def _width_samples(self, width):
        return int(round(width / self.tsamp))

    @timing
    def deredden(self, width, minpts=101, inplace=False):
        """Subtract a running median of `width` seconds, computed on a scrunched
        copy with >= minpts samples per window (time_series.py:93-122)."""
        out = libcpp.deredden_normalise(self.data, self._width_samples(width), minpts,
                                        deredden=True, normalise=False)
        if inplace:
            self._data = out
        else:
            return TimeSeries(out, self.tsamp, metadata=self.metadata)

    def deredden_normalise(self, width, minpts=101):
        """deredden() then normalise() in one device round trip."""
        out = libcpp.deredden_normalise(self.data, self._width_samples(width), minpts,
                                        deredden=True, normalise=True)
        return TimeSeries(out, self.tsamp, metadata=self.metadata)

    def downsample(self, factor, inplace=False):
        """Downsample by a real-valued factor (time_series.py:124-145)."""
        if inplace:
            self._data = downsample(self.data, factor)
            self._tsamp *= factor
        else:
            return TimeSeries(downsample(self.data, factor), factor * self.tsamp, metadata=self.metadata)

    @classmethod
    def generate(cls, length, tsamp, period, phi0=0.5, ducy=0.02, amplitude=10.0, stdnoise=1.0):
        """Noisy von Mises pulse train (time_series.py:170-218)."""
        nsamp = int(round(length / tsamp))
        data = generate_signal(nsamp, period / tsamp, phi0=phi0, ducy=ducy, amplitude=amplitude,
                               stdnoise=stdnoise)
        metadata = Metadata({
            "source_name": "fake",
            "signal_shape": "Von Mises",
            "signal_period": period,
            "signal_initial_phase": phi0,
            "signal_duty_cycle": ducy,
        })
        return cls(data, tsamp, copy=False, metadata=metadata)

    @classmethod
    def from_numpy_array(cls, array, tsamp, copy=False):
        return cls(array, tsamp, copy=copy)

    @classmethod
    @timing
    def from_sigproc(cls, fname, extra_keys={}):
        """SIGPROC dedispersed time series, 8-bit (signedness from the 'signed'
        header key) or 32-bit float (time_series.py:320-362)."""
        from .reading import read_sigproc
        data, meta, tsamp = read_sigproc(fname, extra_keys=extra_keys)
        return cls(data, tsamp, metadata=meta)

    @classmethod
    @timing
    def from_presto_inf(cls, fname):
        """PRESTO .inf + .dat pair (time_series.py:283-318)."""
        from .reading import read_presto
        data, meta, tsamp = read_presto(fname)
        return cls(data, tsamp, metadata=meta)

    @classmethod
    def from_binary(cls, fname, tsamp, dtype=np.float32):
        return cls(np.fromfile(fname, dtype=dtype), tsamp, copy=False)

    @classmethod
    def from_npy_file(cls, fname, tsamp):
        return cls(np.load(fname), tsamp, copy=False)

    @property
    def nsamp(self):
        return self.data.size

    @property
    def length(self):
        return self.nsamp * self.tsamp

    @property
    def tobs(self):
        return self.length

    def __str__(self):
        return "{} {{nsamp = {:d}, tsamp = {:.4e}, tobs = {:.3f}}}".format(
            type(self).__name__, self.nsamp, self.tsamp, self.length)

    __repr__ = __str__

    @classmethod
    def from_dict(cls, items):
        return cls(items["data"], items["tsamp"], metadata=items["metadata"], copy=False)

    def to_dict(self):
        return {"data": self.data, "tsamp": self.tsamp, "metadata": self.metadata}
