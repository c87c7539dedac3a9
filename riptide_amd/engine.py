"""Device-resident, batched hot path (the part bench.py and the multi-GPU
dispatcher drive).  Buffers are torch tensors on the ROCm device; all compute
is the engine's HIP kernels (rt_plan_* / rt_periodogram_device /
rt_deredden_normalise_device in include/riptide_amd.h).
"""
import ctypes

import numpy as np

from . import _lib
from .ffautils import generate_width_trials

_L = _lib.load()
_check = _lib.check


def _stream_handle(stream=None):
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


class PeriodogramPlan:
    """Compiled periodogram plan for series of `size` samples: downsampling
    ladder, trial grid and the cone-kernel pass schedule (host-built once,
    uploaded to the current device)."""

    def __init__(self, size, tsamp, widths, period_min, period_max, bins_min, bins_max, device=None):
        import torch
        dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        _check(_L.rt_set_device(dev.index))
        self.device = dev
        self.size, self.tsamp = int(size), float(tsamp)
        self.widths = np.ascontiguousarray(widths, dtype=np.uint64)
        self.period_min, self.period_max = float(period_min), float(period_max)
        self.bins_min, self.bins_max = int(bins_min), int(bins_max)
        h = ctypes.c_void_p()
        with torch.cuda.device(dev):
            _check(_L.rt_plan_create(self.size, self.tsamp, _lib.ptr(self.widths), self.widths.size,
                                     self.period_min, self.period_max, self.bins_min, self.bins_max,
                                     ctypes.byref(h)))
        self._h = h
        L, W = ctypes.c_size_t(), ctypes.c_size_t()
        _check(_L.rt_plan_shape(h, ctypes.byref(L), ctypes.byref(W)))
        self.length, self.num_widths = L.value, W.value
        self._grid = None

    @classmethod
    def for_search(cls, size, tsamp, period_min, period_max, bins_min=240, bins_max=260, ducy_max=0.2,
                   wtsp=1.5, device=None):
        widths = generate_width_trials(bins_min, ducy_max=ducy_max, wtsp=wtsp)
        return cls(size, tsamp, widths, period_min, period_max, bins_min, bins_max, device=device)

    def grid(self):
        """(periods f64[L], foldbins u32[L]) -- bit-exact with the reference."""
        if self._grid is None:
            periods = np.empty(self.length, dtype=np.float64)
            foldbins = np.empty(self.length, dtype=np.uint32)
            _check(_L.rt_plan_grid(self._h, _lib.ptr(periods), _lib.ptr(foldbins)))
            self._grid = (periods, foldbins)
        return self._grid

    def workspace_bytes(self, batch):
        b = ctypes.c_size_t()
        _check(_L.rt_plan_workspace_bytes(self._h, int(batch), ctypes.byref(b)))
        return b.value

    def stats(self):
        u = [ctypes.c_uint64() for _ in range(4)]
        d = [ctypes.c_double() for _ in range(2)]
        _check(_L.rt_plan_stats(self._h, *(ctypes.byref(x) for x in u[:3]), ctypes.byref(d[0]),
                                ctypes.byref(d[1]), ctypes.byref(u[3])))
        return {"transforms": u[0].value, "items": u[1].value, "launches": u[2].value,
                "alg_bytes": d[0].value, "moved_bytes": d[1].value, "cells": u[3].value}

    def run(self, data, out=None, workspace=None, stream=None, check=False):
        """S/N of a batch of series: data float32 [B, size] (or [size]) on the
        device -> float32 [B, L, W].  Stream-ordered; no host synchronisation
        unless `check` (then the plan's device error flag is read: see
        check()).  Allocations happen on `stream` (default: the current one)."""
        import torch
        squeeze = data.dim() == 1
        if squeeze:
            data = data.unsqueeze(0)
        if data.dim() != 2 or data.dtype != torch.float32 or data.device != self.device or data.shape[1] != self.size:
            raise ValueError("data must be float32 [B, size] on the plan's device")
        if data.stride(1) != 1:
            raise ValueError("data rows must be contiguous")
        B = data.shape[0]
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        with torch.cuda.stream(s):
            if out is None:
                out = torch.empty((B, self.length, self.num_widths), dtype=torch.float32, device=self.device)
            elif (out.dtype != torch.float32 or out.device != self.device or not out.is_contiguous()
                  or tuple(out.shape) != (B, self.length, self.num_widths)):
                raise ValueError(f"out must be a contiguous float32 [{B}, {self.length}, {self.num_widths}] "
                                 "tensor on the plan's device")
            need = self.workspace_bytes(B)
            if workspace is None:
                workspace = torch.empty(need, dtype=torch.uint8, device=self.device)
            elif (workspace.dtype != torch.uint8 or workspace.device != self.device or not workspace.is_contiguous()
                  or workspace.numel() < need):
                raise ValueError(f"workspace must be a contiguous uint8 tensor of >= {need} bytes on the plan's device")
            _check(_L.rt_periodogram_device(self._h, _lib.ptr(data), B, data.stride(0), _lib.ptr(out),
                                            self.length * self.num_widths, _lib.ptr(workspace), workspace.numel(),
                                            _stream_handle(s)))
        if check:
            self.check(s)
        return out[0] if squeeze else out

    def _ws_ok(self, workspace, B):
        import torch
        need = self.workspace_bytes(B)
        if (workspace is None or workspace.dtype != torch.uint8 or workspace.device != self.device
                or not workspace.is_contiguous() or workspace.numel() < need):
            raise ValueError(f"workspace must be a contiguous uint8 tensor of >= {need} bytes on the plan's device")

    def ladder(self, data, workspace, stream=None):
        """First half of run(): the downsampling ladder of data float32 [B, size]
        into `workspace`'s leaf buffer (rt_periodogram_ladder_device).  With
        passes() on another stream, batch k + 1's ladder overlaps batch k's
        FFA passes; the caller orders the two halves of one batch (an event)
        and keeps a workspace per batch in flight."""
        import torch
        if data.dim() != 2 or data.dtype != torch.float32 or data.device != self.device or data.shape[1] != self.size:
            raise ValueError("data must be float32 [B, size] on the plan's device")
        if data.stride(1) != 1:
            raise ValueError("data rows must be contiguous")
        B = data.shape[0]
        self._ws_ok(workspace, B)
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        _check(_L.rt_periodogram_ladder_device(self._h, _lib.ptr(data), B, data.stride(0), _lib.ptr(workspace),
                                               workspace.numel(), _stream_handle(s)))

    def passes(self, out, workspace, stream=None):
        """Second half of run(): FFA passes + fused S/N of the batch whose
        ladder filled `workspace`, into out float32 [B, L, W]."""
        import torch
        B = out.shape[0]
        if (out.dtype != torch.float32 or out.device != self.device or not out.is_contiguous()
                or tuple(out.shape) != (B, self.length, self.num_widths)):
            raise ValueError(f"out must be a contiguous float32 [B, {self.length}, {self.num_widths}] "
                             "tensor on the plan's device")
        self._ws_ok(workspace, B)
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        _check(_L.rt_periodogram_passes_device(self._h, B, _lib.ptr(out), self.length * self.num_widths,
                                               _lib.ptr(workspace), workspace.numel(), _stream_handle(s)))
        return out

    def check(self, stream=None):
        """Raise EngineError if any cone work unit of the runs since the last
        check broke its LDS / register budget (its S/N rows were left
        unwritten).  Synchronises `stream` (default: the current stream)."""
        _check(_L.rt_plan_check(self._h, _stream_handle(stream)))

    def __del__(self, _destroy=_L.rt_plan_destroy):
        # the default argument keeps the function alive through interpreter
        # shutdown, when module globals may already be cleared
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            _destroy(h)
            self._h = None


def deredden_workspace_bytes(size, width_samples, min_points, batch):
    b = ctypes.c_size_t()
    _check(_L.rt_deredden_workspace_bytes(int(size), int(width_samples), int(min_points), int(batch),
                                          ctypes.byref(b)))
    return b.value


def deredden_normalise(data, width_samples, min_points=101, deredden=True, normalise=True, out=None,
                       workspace=None, stream=None):
    """TimeSeries.deredden(...).normalise() for a batch [B, N] of device series."""
    import torch
    squeeze = data.dim() == 1
    if squeeze:
        data = data.unsqueeze(0)
    if data.dim() != 2 or data.dtype != torch.float32 or data.device.type != "cuda" or data.stride(1) != 1:
        raise ValueError("data must be float32 [B, N] device rows with unit stride")
    B, N = data.shape
    s = stream if stream is not None else torch.cuda.current_stream(data.device)
    with torch.cuda.stream(s):
        if out is None:
            out = torch.empty((B, N), dtype=torch.float32, device=data.device)
        elif (out.dim() != 2 or tuple(out.shape) != (B, N) or out.dtype != torch.float32
              or out.device != data.device or out.stride(1) != 1):
            raise ValueError("out must be float32 [B, N] rows with unit stride on the data's device")
        need = deredden_workspace_bytes(N, width_samples, min_points, B)
        if workspace is None:
            workspace = torch.empty(need, dtype=torch.uint8, device=data.device)
        elif (workspace.dtype != torch.uint8 or workspace.device != data.device or not workspace.is_contiguous()
              or workspace.numel() < need):
            raise ValueError(f"workspace must be a contiguous uint8 tensor of >= {need} bytes on the data's device")
        _check(_L.rt_deredden_normalise_device(_lib.ptr(data), N, B, data.stride(0), int(width_samples),
                                               int(min_points), int(bool(deredden)), int(bool(normalise)),
                                               _lib.ptr(out), out.stride(0), _lib.ptr(workspace), workspace.numel(),
                                               _stream_handle(s)))
    return out[0] if squeeze else out


def profile_enable(on=True):
    _check(_L.rt_profile_enable(int(bool(on))))


def profile_reset():
    _check(_L.rt_profile_reset())


def profile_read(kind=0):
    """Accumulated (ms, algorithmic bytes, moved bytes, launches) of the cone
    kernel (kind 0) or the downsample ladder (kind 1) since the last reset."""
    ms, alg, mv, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_double(), ctypes.c_uint64()
    _check(_L.rt_profile_read(int(kind), ctypes.byref(ms), ctypes.byref(alg), ctypes.byref(mv), ctypes.byref(n)))
    return {"ms": ms.value, "alg_bytes": alg.value, "moved_bytes": mv.value, "launches": n.value}
