"""Host logic of the device find_peaks (riptide_amd/peaks.py), checked on the
CPU: numpy's 'linear' percentile rebuilt from order statistics, and the
padded threshold polynomial, must equal numpy's own results bit for bit
(peak_detection.py:81-83, 123-131)."""
import numpy as np
import pytest

pytestmark = pytest.mark.filterwarnings("ignore::RuntimeWarning")


def _peaks():
    # riptide_amd.peaks imports the engine library (loads without a GPU)
    from riptide_amd import peaks
    return peaks


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 7, 10, 97, 1246, 1248, 4096])
def test_percentiles_from_order_stats_bit_exact(n):
    P = _peaks()
    rng = np.random.RandomState(n)
    segs = rng.normal(size=(33, n)).astype(np.float32)
    segs[3, :] = 1.5                                   # ties
    segs[5, : n // 2] = -0.0
    ranks, gamma = P.percentile_ranks(n)
    srt = np.sort(segs, axis=1)
    stats = srt[:, ranks]                              # what the device returns
    got = P.percentiles_from_order_stats(stats, gamma)
    ref = np.percentile(segs.astype(float), (25, 50, 75), axis=-1)
    for k in range(3):
        assert np.array_equal(got[k].view(np.int64), ref[k].view(np.int64))


def test_percentiles_nan_segment():
    P = _peaks()
    segs = np.random.RandomState(1).normal(size=(4, 50)).astype(np.float32)
    segs[2, 7] = np.nan
    ranks, gamma = P.percentile_ranks(50)
    stats = np.sort(segs, axis=1)[:, ranks]
    stats[2, :] = np.nan                               # device: NaN for a segment holding a NaN
    got = P.percentiles_from_order_stats(stats, gamma)
    ref = np.percentile(segs.astype(float), (25, 50, 75), axis=-1)
    for k in range(3):
        assert np.array_equal(got[k], ref[k], equal_nan=True)


def test_padded_polynomial_value():
    # the device evaluates Horner over leading-zero-padded coefficients
    rng = np.random.RandomState(3)
    x = np.log(rng.uniform(0.05, 50.0, size=1000))
    for coeffs in ([2.5], [0.0, 1.0], [1e-3, -0.2, 7.0], [0.0, 0.0, 6.0]):
        poly = np.poly1d(coeffs)
        ref = poly(x)
        c = np.zeros(3)
        c[3 - poly.coefficients.size:] = poly.coefficients
        y = np.zeros_like(x)
        for pv in c:
            y = y * x + pv
        assert np.array_equal(y, ref)
