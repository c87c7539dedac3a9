"""ctypes loader of the engine's C ABI (include/riptide_amd.h).

The shared library is built in-tree (``make -C riptide_amd/csrc``, or
``__graft_entry__.build()``) and loaded from this package directory.  There is
no fallback: if the library is missing or fails to load, importing the compute
API raises, loudly.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RIPTIDE_AMD_LIB") or os.path.join(_HERE, "libriptide_amd.so")

RT_OK, RT_EINVAL, RT_EHIP, RT_EINTERNAL = 0, 1, 2, 3

_c_sz = ctypes.c_size_t
_c_d = ctypes.c_double
_c_f = ctypes.c_float
_c_i = ctypes.c_int
_vp = ctypes.c_void_p
_psz = ctypes.POINTER(ctypes.c_size_t)
_pd = ctypes.POINTER(ctypes.c_double)
_pu64 = ctypes.POINTER(ctypes.c_uint64)

# name -> (restype, argtypes); pointers are passed as c_void_p (numpy .ctypes.data
# or torch .data_ptr())
_SIGNATURES = {
    "rt_last_error": (ctypes.c_char_p, []),
    "rt_version": (ctypes.c_char_p, []),
    "rt_set_device": (_c_i, [_c_i]),
    "rt_rollback": (_c_i, [_vp, _c_sz, _c_sz, _vp]),
    "rt_fused_rollback_add": (_c_i, [_vp, _vp, _c_sz, _c_sz, _vp]),
    "rt_circular_prefix_sum": (_c_i, [_vp, _c_sz, _c_sz, _vp]),
    "rt_ffa2": (_c_i, [_vp, _c_sz, _c_sz, _vp]),
    "rt_benchmark_ffa2": (_c_i, [_c_sz, _c_sz, _c_sz, _pd]),
    "rt_snr1": (_c_i, [_vp, _c_sz, _vp, _c_sz, _c_f, _vp]),
    "rt_snr2": (_c_i, [_vp, _c_sz, _c_sz, _vp, _c_sz, _c_f, _vp]),
    "rt_downsampled_size": (_c_sz, [_c_sz, _c_d]),
    "rt_downsample": (_c_i, [_vp, _c_sz, _c_d, _vp]),
    "rt_downsample_rows": (_c_i, [_vp, _c_sz, _c_sz, _c_d, _vp]),
    "rt_periodogram_length": (_c_i, [_c_sz, _c_d, _c_d, _c_d, _c_sz, _c_sz, _psz]),
    "rt_periodogram": (_c_i, [_vp, _c_sz, _c_d, _vp, _c_sz, _c_d, _c_d, _c_sz, _c_sz, _vp, _vp, _vp]),
    "rt_running_median": (_c_i, [_vp, _c_sz, _c_sz, _vp]),
    "rt_fast_running_median": (_c_i, [_vp, _c_sz, _c_sz, _c_sz, _vp]),
    "rt_deredden_normalise": (_c_i, [_vp, _c_sz, _c_sz, _c_sz, _c_i, _c_i, _vp]),
    "rt_periodogram_grid": (_c_i, [_c_sz, _c_d, _c_d, _c_d, _c_sz, _c_sz, _vp, _vp]),
    "rt_ffa_schedule_check": (_c_i, [_c_sz, _c_sz, _pu64]),
    "rt_schedule_check": (_c_i, [_c_sz, _c_d, _c_sz, _c_d, _c_d, _c_sz, _c_sz, _pu64, _pu64, _pu64, _pd, _pd,
                                 _pu64]),
    "rt_plan_create": (_c_i, [_c_sz, _c_d, _vp, _c_sz, _c_d, _c_d, _c_sz, _c_sz, _vp]),
    "rt_plan_destroy": (None, [_vp]),
    "rt_plan_shape": (_c_i, [_vp, _psz, _psz]),
    "rt_plan_grid": (_c_i, [_vp, _vp, _vp]),
    "rt_plan_workspace_bytes": (_c_i, [_vp, _c_sz, _psz]),
    "rt_periodogram_device": (_c_i, [_vp, _vp, _c_sz, _c_sz, _vp, _c_sz, _vp, _c_sz, _vp]),
    "rt_periodogram_ladder_device": (_c_i, [_vp, _vp, _c_sz, _c_sz, _vp, _c_sz, _vp]),
    "rt_periodogram_passes_device": (_c_i, [_vp, _c_sz, _vp, _c_sz, _vp, _c_sz, _vp]),
    "rt_plan_check": (_c_i, [_vp, _vp]),
    "rt_deredden_workspace_bytes": (_c_i, [_c_sz, _c_sz, _c_sz, _c_sz, _psz]),
    "rt_deredden_normalise_device": (_c_i, [_vp, _c_sz, _c_sz, _c_sz, _c_sz, _c_sz, _c_i, _c_i, _vp, _c_sz,
                                            _vp, _c_sz, _vp]),
    "rt_profile_enable": (_c_i, [_c_i]),
    "rt_profile_read": (_c_i, [_c_i, _pd, _pd, _pd, _pu64]),
    "rt_profile_reset": (_c_i, []),
    "rt_diag_stamps": (_c_i, [_pu64, _c_i]),
    "rt_diag_timeline": (_c_i, [_pu64, ctypes.c_uint64, _pu64]),
    "rt_diag_launches": (_c_i, [_pu64, ctypes.c_uint64, _pu64]),
    "rt_plan_stats": (_c_i, [_vp, _pu64, _pu64, _pu64, _pd, _pd, _pu64]),
    "rt_convert_samples_device": (_c_i, [_vp, _c_sz, _c_i, _vp, _vp]),
    "rt_segment_order_stats_device": (_c_i, [_vp, _c_sz, _c_sz, _c_sz, _c_sz, _c_sz, _c_sz, _vp, _c_sz, _vp, _vp]),
    "rt_threshold_select_device": (_c_i, [_vp, _c_sz, _c_sz, _c_sz, _c_sz, _vp, _vp, _c_sz, _c_d, _vp, _vp, _c_sz,
                                          _vp]),
    "rt_ladder_check": (_c_i, [_c_sz, _c_d, _c_d, _c_d, _c_sz, _c_sz, ctypes.POINTER(_c_i), _pu64]),
}

EXPORTED = tuple(_SIGNATURES)

# test build only (libriptide_amd_testhooks.so, include/riptide_amd_test.h);
# bound when the loaded library has them
_TEST_SIGNATURES = {
    "rt_test_corrupt_next_plans": (_c_i, [_c_i]),
}
TESTHOOKS_PATH = os.path.join(_HERE, "libriptide_amd_testhooks.so")

_lib = None


class EngineError(RuntimeError):
    """A HIP runtime or internal failure inside the engine."""


def load():
    """Load (once) and return the engine library.  Raises ImportError if absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"riptide_amd engine library not found at {LIB_PATH}; build it with "
            "`make -C riptide_amd/csrc` or `python -c 'import __graft_entry__ as g; g.build()'`")
    # One HIP runtime per process: torch ships its own libamdhip64, and an
    # engine library loaded before torch binds /opt/rocm's instead -- the
    # engine's launches then fail with "no ROCm-capable device is detected"
    # once torch initialises its runtime (`import riptide_amd; import torch`).
    # Importing torch first makes the engine resolve to torch's runtime.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    # The plan pointer is opaque: rt_plan_create takes an rt_plan** (void*)
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_LOCAL)
    for name, (res, args) in _SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    for name, (res, args) in _TEST_SIGNATURES.items():
        if hasattr(lib, name):
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
    _lib = lib
    return lib


def check(rc):
    """Map an RT_* return code to the reference's exception types."""
    if rc == RT_OK:
        return
    msg = _lib.rt_last_error().decode("utf-8", "replace")
    if rc == RT_EINVAL:
        raise ValueError(msg)
    raise EngineError(msg)


def ptr(a):
    """Raw address of a numpy array or torch tensor."""
    if hasattr(a, "data_ptr"):
        return ctypes.c_void_p(a.data_ptr())
    return ctypes.c_void_p(a.ctypes.data)
