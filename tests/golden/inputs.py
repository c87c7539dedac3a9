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


# ---------------------------------------------------------------- end-to-end known answers
# riptide/tests/presto_generation.py:31-58 + test_rseek.py:31-54: np.random.seed(0),
# TimeSeries.generate(128 s, 256 us, P = 1 s, amplitude 20, ducy 0.02), PRESTO
# format, rseek options Pmin 0.5, Pmax 2, bmin 480, bmax 520, smin 7 (others
# at rseek's defaults: rmed_width 4, rmed_minpts 101, wtsp 1.5, clrad 0.2;
# ffa_search(ducy_max=0.3)).
RSEEK_CASE = dict(tobs=128.0, tsamp=256e-6, period=1.0, amplitude=20.0, ducy=0.02, dm=0.0,
                  pmin=0.5, pmax=2.0, bmin=480, bmax=520, smin=7.0, rmed_width=4.0, rmed_minpts=101,
                  wtsp=1.5, clrad=0.2, ducy_max=0.3)

# riptide/tests/test_pipeline.py:39-74 with pipeline_config_A.yml: three DM
# trials (dm, amplitude, ducy), each generated after np.random.seed(0).
PIPELINE_CASE = dict(
    tobs=128.0, tsamp=256e-6, period=1.0,
    trials=[(0.0, 10.0, 0.05), (10.0, 20.0, 0.02), (20.0, 10.0, 0.05)],
    dereddening={"rmed_width": 5.0, "rmed_minpts": 101},
    ranges=[
        {"name": "medium",
         "ffa_search": {"period_min": 0.5, "period_max": 4.0, "bins_min": 480, "bins_max": 520, "fpmin": 8,
                        "wtsp": 1.5},
         "find_peaks": {"smin": 7.0}},
        {"name": "long",
         "ffa_search": {"period_min": 4.0, "period_max": 120.0, "bins_min": 960, "bins_max": 1040, "fpmin": 8,
                        "wtsp": 1.5},
         "find_peaks": {"smin": 7.0}},
    ],
    clustering_radius=0.2,
)


def generated_series(tobs, tsamp, period, amplitude, ducy, generate_signal):
    """TimeSeries.generate (time_series.py:170-218) after np.random.seed(0),
    as float32 (what presto_generation.py writes to the .dat file).
    `generate_signal` is the implementation under test's (or the reference's)
    libffa.generate_signal; numpy's legacy global RNG supplies the noise."""
    np.random.seed(0)
    nsamp = int(round(tobs / tsamp))
    return np.asarray(generate_signal(nsamp, period / tsamp, phi0=0.5, ducy=ducy, amplitude=amplitude,
                                      stdnoise=1.0), dtype=np.float32)


# The fused downsampling ladder's margin edge (kDsFusedMargin = 512 floats):
# two rungs, f = 452.9 and 509.5125 (ceil(f) + 2 = 512, the largest window
# the fused kernel stages), 16-17 bins.
LADDER_EDGE_CASE = dict(n=1 << 20, tsamp=1e-3, pmin=452.9 * 1e-3 * 16, pmax=452.9 * 1e-3 * 16 * 1.125 ** 2 * 0.999,
                        bmin=16, bmax=17, ducy_max=0.2)


# ---------------------------------------------------------------- cfg5: rffa beam of SIGPROC files
# BASELINE.json configs[4] at reduced trial count: 2^23-sample SIGPROC .tim
# DM trials @ 64 us (537 s, "SUPERB-like"), refdm = 10 k, searched with
# riptide's example pipeline configuration (pipeline/config/example.yaml:
# dereddening 5 s / 101 points; ranges short 0.2-0.5 s @ 240-260 bins, medium
# 0.5-2 s @ 480-520, long 2-120 s @ 960-1040; smin 6).  Two top-hat pulsars
# whose amplitude peaks at DM 40 (P = 0.7137 s) and DM 20 (P = 3.1416 s);
# trials 6 and 7 are 8-bit files (unsigned / signed).
CFG5 = dict(
    n=1 << 23, tsamp=64e-6, nfiles=8,
    dereddening={"rmed_width": 5.0, "rmed_minpts": 101},
    ranges=[
        {"name": "short",
         "ffa_search": {"period_min": 0.2, "period_max": 0.5, "bins_min": 240, "bins_max": 260, "fpmin": 8,
                        "wtsp": 1.5},
         "find_peaks": {"smin": 6.0}},
        {"name": "medium",
         "ffa_search": {"period_min": 0.5, "period_max": 2.0, "bins_min": 480, "bins_max": 520, "fpmin": 8,
                        "wtsp": 1.5},
         "find_peaks": {"smin": 6.0}},
        {"name": "long",
         "ffa_search": {"period_min": 2.0, "period_max": 120.0, "bins_min": 960, "bins_max": 1040, "fpmin": 8,
                        "wtsp": 1.5},
         "find_peaks": {"smin": 6.0}},
    ],
    chunksize=4,
)


def cfg5_trial(k, n=None):
    """(stored samples, SIGPROC header) of cfg5 DM trial k.  Stored dtype:
    float32, or uint8 / int8 for trials 6 / 7 (what a reader hands over)."""
    c = CFG5
    n = c["n"] if n is None else n
    tsamp = c["tsamp"]
    dm = 10.0 * k
    rs = np.random.RandomState(700 + k)
    x = rs.normal(size=n)
    walk = np.cumsum(rs.normal(size=n // 8192 + 1)) * 0.5
    x = x + np.repeat(walk, 8192)[:n]
    a1 = 30.0 * max(0.0, 1.0 - abs(dm - 40.0) / 25.0)
    a2 = 22.0 * max(0.0, 1.0 - abs(dm - 20.0) / 25.0)
    if a1:
        x = x + tophat_train(n, tsamp, 0.7137, ducy=0.03, amplitude=a1)
    if a2:
        x = x + tophat_train(n, tsamp, 3.1416, ducy=0.02, amplitude=a2, phi0=0.6)
    hdr = {"source_name": f"cfg5_DM{dm:.1f}", "tsamp": tsamp, "tstart": 60000.0, "src_raj": 123456.7,
           "src_dej": -301502.5, "nchans": 1, "refdm": dm}
    if k == 6:
        data = np.clip(np.round(x * 10.0 + 128.0), 0, 255).astype(np.uint8)
        hdr.update(nbits=8, signed=False)
    elif k == 7:
        data = np.clip(np.round(x * 10.0), -128, 127).astype(np.int8)
        hdr.update(nbits=8, signed=True)
    else:
        data = x.astype(np.float32)
        hdr.update(nbits=32)
    return data, hdr
