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


def test_cluster_peaks_pipeline_order():
    """clustering.cluster_peaks restates Pipeline.search's sort and
    Pipeline.cluster_peaks (pipeline.py:186, 192-215): peaks sorted by
    increasing period (stable: equal periods keep their input order), then
    friends-of-friends in frequency at radius / Tobs -- a known answer with a
    chain whose ends are more than one radius apart (one cluster), a gap of
    exactly the radius (linked) and a tie in period."""
    from riptide_amd.clustering import cluster_peaks
    from riptide_amd.peak_detection import Peak
    tobs, rad = 100.0, 0.2                 # radius 0.002 Hz
    freqs = [1.0, 1.0015, 1.003, 1.0045,   # a chain: 0.0015 Hz steps, 0.0045 end to end
             2.0, 2.002,                   # linked at exactly the radius
             3.0, 3.0021,                  # split: 0.0021 > 0.002
             0.5, 0.5]                     # a tie in period
    peaks = [Peak(1.0 / f, f, 3, 0.01, 1, i, 10.0 + i, 5.0 * i) for i, f in enumerate(freqs)]
    rs = np.random.RandomState(3)
    shuffled = [peaks[i] for i in rs.permutation(len(peaks))]
    ps, clusters = cluster_peaks([tuple(p) for p in shuffled], rad, tobs)
    assert [p.period for p in ps] == sorted(p.period for p in peaks)
    ties = [p.ip for p in ps if p.freq == 0.5]
    assert ties == [p.ip for p in shuffled if p.freq == 0.5]          # stable sort
    got = sorted(sorted(p.ip for p in cl) for cl in clusters)
    assert got == [[0, 1, 2, 3], [4, 5], [6], [7], [8, 9]]
    assert cluster_peaks([], rad, tobs) == ([], [])


def test_polyfit_columns_bit_exact():
    """peaks.polyfit_columns / poly1d_coefficients == np.poly1d(np.polyfit(x,
    y, deg)).coefficients for every row, bit for bit (the threshold polynomial
    of find_peaks, peak_detection.py:187-199): segment counts of the
    BASELINE / cfg5 ranges, float32 and float64 rows, exact-zero leading
    coefficients (a constant and a linear row)."""
    from riptide_amd.peaks import poly1d_coefficients, polyfit_columns
    rng = np.random.default_rng(5)
    for nseg in (10, 11, 53, 97, 400):
        x = np.log(np.sort(rng.uniform(0.008, 12.0, nseg)))
        for dtype in (np.float64, np.float32):
            Y = rng.normal(7.0, 0.6, (37, nseg)).astype(dtype)
            Y[0] = 6.5                                   # constant: leading coefficients ~0
            Y[1] = (2.0 * x + 1.0).astype(dtype)         # linear
            got = polyfit_columns(x, Y, 2)
            for k in range(Y.shape[0]):
                want = np.poly1d(np.polyfit(x, Y[k], 2)).coefficients
                assert np.array_equal(poly1d_coefficients(got[k]), want), (nseg, dtype, k)
    assert np.array_equal(poly1d_coefficients([0.0, 0.0, 3.0]), np.poly1d([0.0, 0.0, 3.0]).coefficients)
    assert np.array_equal(poly1d_coefficients([0.0]), np.poly1d([0.0]).coefficients)


def test_poly1d_table_matches_per_fit():
    """peaks.poly1d_table (every (trial, width) at once) == the per-fit
    np.poly1d coefficients and their right-aligned, zero-padded table rows,
    including leading zeros of both signs and all-zero fits."""
    from riptide_amd.peaks import poly1d_coefficients, poly1d_table
    rng = np.random.default_rng(11)
    fits = rng.normal(0.0, 1.0, (5, 7, 3))
    fits[0, 0] = [0.0, 0.0, 4.0]
    fits[0, 1] = [-0.0, 2.0, 1.0]
    fits[0, 2] = [0.0, -0.0, 0.0]
    fits[1, 3] = [0.0, 0.0, -0.0]
    fits[2, 4] = [1.0, 0.0, 0.0]
    fits[3, 5] = [-0.0, 0.0, 5.0]
    coeffs, polycos = poly1d_table(fits)
    for b in range(fits.shape[0]):
        for iw in range(fits.shape[1]):
            want = np.poly1d(fits[b, iw]).coefficients
            assert np.array_equal(polycos[b][iw], want) and polycos[b][iw].dtype == want.dtype
            row = np.zeros(3)
            c = poly1d_coefficients(want)
            row[3 - c.size:] = c
            assert np.array_equal(coeffs[b, iw], row) and not np.signbit(coeffs[b, iw][:3 - c.size]).any()
