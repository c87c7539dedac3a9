"""Deterministic inputs for the golden vectors and the parity tests.

Every input is regenerated from np.random.RandomState(seed) (stream-stable
across numpy versions) plus IEEE-exact arithmetic, so the same bytes appear in
the build container (where make_golden.py ran the reference) and on the GPU
box.  Each golden record also stores the sha256 of its input so a mismatch is
reported as such rather than as a parity failure.
"""
import numpy as np

# Hand-computed 8x8 known answer of the reference test suite
# (riptide/tests/test_ffa_base_functions.py:12-32): a one-bin pulse in the last
# column; the transform is also invariant under phase rotation.
FFA_IN_88 = np.zeros((8, 8), dtype=np.float32)
FFA_IN_88[:, 7] = 1.0
FFA_OUT_88 = np.array([
    [0, 0, 0, 0, 0, 0, 0, 8],
    [0, 0, 0, 0, 0, 0, 4, 4],
    [0, 0, 0, 0, 0, 2, 4, 2],
    [0, 0, 0, 0, 2, 2, 2, 2],
    [0, 0, 0, 1, 2, 2, 2, 1],
    [0, 0, 1, 2, 1, 1, 2, 1],
    [0, 1, 1, 1, 2, 1, 1, 1],
    [1, 1, 1, 1, 1, 1, 1, 1]], dtype=np.float32)

# (rows, cols, seed): tiny/odd shapes, BASELINE-like shapes, LDS edge shapes
FFA_CASES = [
    (1, 9, 1), (2, 7, 2), (3, 5, 3), (5, 3, 4), (8, 8, 5), (37, 17, 6), (129, 260, 7),
    (1000, 250, 8), (4097, 33, 9), (9001, 16, 10), (20000, 16, 11), (2500, 1200, 12),
]
DS_FACTORS = [1.0000001, 1.6276, 2.5, 7.3, 16.0, 40.1, 162.76, 20000.0]
SNR_WIDTHS = [1, 2, 3, 4, 6, 9, 13, 19, 28, 42]
RMED_WIDTHS = [1, 3, 5, 7, 11, 25, 37, 101, 999]
FAST_RMED_CASES = [(15625, 101), (1001, 101), (31, 101), (7813, 51)]


def noise(n, seed):
    return np.random.RandomState(seed).normal(size=n).astype(np.float32)


def ffa_block(m, p, seed):
    return np.random.RandomState(seed).normal(size=(m, p)).astype(np.float32)


def tophat_train(n, tsamp, period, ducy=0.02, amplitude=15.0, phi0=0.3):
    """Unit-L2 top-hat pulse train scaled by `amplitude` (float64), built from
    IEEE-exact operations only (no transcendental functions)."""
    t = np.arange(n, dtype=np.float64) * tsamp
    phase = np.mod(t / period + phi0, 1.0)
    on = phase < ducy
    k = int(on.sum())
    s = np.zeros(n, dtype=np.float64)
    if k:
        s[on] = amplitude / np.sqrt(float(k))
    return s


def with_signal(n, tsamp, seed, period, amplitude):
    x = np.random.RandomState(seed).normal(size=n)
    if amplitude:
        x = x + tophat_train(n, tsamp, period, amplitude=amplitude)
    return x.astype(np.float32)


# Reduced-size periodograms on the BASELINE configs' search parameters
PGRAM_CASES = [
    dict(name="cfg1", n=1 << 16, tsamp=256e-6, pmin=0.5, pmax=2.0, bmin=240, bmax=260, ducy_max=0.2, seed=21, period=1.0, amp=15.0),
    dict(name="cfg2", n=1 << 15, tsamp=256e-6, pmin=0.1, pmax=10.0, bmin=240, bmax=260, ducy_max=0.05, seed=22, period=0.33, amp=15.0),
    dict(name="cfg3", n=1 << 15, tsamp=256e-6, pmin=0.2, pmax=5.0, bmin=240, bmax=260, ducy_max=0.2, seed=23, period=0.7, amp=15.0),
    dict(name="cfg4", n=1 << 16, tsamp=64e-6, pmin=0.002, pmax=0.5, bmin=16, bmax=32, ducy_max=0.2, seed=24, period=0.0123, amp=15.0),
    dict(name="nods", n=1 << 16, tsamp=1e-3, pmin=0.8, pmax=1.2, bmin=800, bmax=1200, ducy_max=0.2, seed=25, period=1.0, amp=20.0),
    dict(name="rseek", n=1 << 16, tsamp=256e-6, pmin=0.5, pmax=2.0, bmin=480, bmax=520, ducy_max=0.2, seed=26, period=1.0, amp=15.0),
]


def pgram_input(case):
    return with_signal(case["n"], case["tsamp"], case["seed"], case["period"], case["amp"])


# Reduced-size full ffa_search (deredden + normalise + periodogram + find_peaks)
SEARCH_CASES = [
    dict(name="s1", n=1 << 17, tsamp=256e-6, pmin=0.5, pmax=2.0, bmin=240, bmax=260, ducy_max=0.2,
         rmed_width=4.0, rmed_minpts=101, seed=31, period=1.0, amp=20.0, red=2.0),
    dict(name="s4", n=1 << 16, tsamp=64e-6, pmin=0.002, pmax=0.5, bmin=16, bmax=32, ducy_max=0.2,
         rmed_width=0.5, rmed_minpts=101, seed=34, period=0.0123, amp=20.0, red=1.0),
]


def search_input(case):
    """Signal + white noise + a slow sinusoid-free red-noise ramp (a random walk
    of the RandomState stream), offset so dereddening has work to do."""
    n = case["n"]
    rs = np.random.RandomState(case["seed"])
    x = rs.normal(size=n)
    walk = np.cumsum(rs.normal(size=n // 4096 + 1)) * case["red"]
    x = x + np.repeat(walk, 4096)[:n] + 3.0
    x = x + tophat_train(n, case["tsamp"], case["period"], amplitude=case["amp"])
    return x.astype(np.float32)


# Full-size BASELINE configurations (BASELINE.json "configs")
FULL_CASES = [
    dict(name="cfg1", n=2343750, tsamp=256e-6, pmin=0.5, pmax=2.0, bmin=240, bmax=260, ducy_max=0.2, seed=0, period=1.0, amp=20.0),
    dict(name="cfg2", n=1 << 23, tsamp=256e-6, pmin=0.1, pmax=10.0, bmin=240, bmax=260, ducy_max=0.05, seed=2, period=3.3, amp=14.0),
    dict(name="cfg3", n=1 << 22, tsamp=256e-6, pmin=0.2, pmax=5.0, bmin=240, bmax=260, ducy_max=0.2, seed=0, period=1.234, amp=15.0),
    dict(name="cfg4", n=1 << 22, tsamp=64e-6, pmin=0.002, pmax=0.5, bmin=16, bmax=32, ducy_max=0.2, seed=4, period=0.0123, amp=15.0),
]


def full_input(case):
    return with_signal(case["n"], case["tsamp"], case["seed"], case["period"], case["amp"])


def trial_input(k, n=1 << 22, tsamp=256e-6):
    """cfg3 batch trial k: white noise from RandomState(k); every 64th trial
    carries a pulsar (period in 0.2-5 s, amplitude 10-20, drawn from the same
    stream after the noise) -- SURVEY.md §8(d)."""
    rs = np.random.RandomState(k)
    x = rs.normal(size=n)
    if k % 64 == 0:
        period = rs.uniform(0.2, 5.0)
        amp = rs.uniform(10.0, 20.0)
        x = x + tophat_train(n, tsamp, period, amplitude=amp)
    return x.astype(np.float32)


def sample_rows(length, count=500, seed=123):
    count = min(count, length)
    return np.sort(np.random.RandomState(seed).choice(length, size=count, replace=False))
