"""Pin the CPU oracle (oracle/ffa_oracle.c + oracle/oracle.py) against golden
vectors produced by the reference implementation itself (make_golden.py).

Bit-exact: FFA transform, period grid, fold bins, running median.
1e-4 relative (BASELINE.json): S/N, since the reference build's -ffast-math
reorders float sums (SURVEY.md §0 finding 3).
"""
import hashlib

import numpy as np
import pytest

import inputs
from conftest import snr_close


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_ffa_known_answer_88(oracle, golden):
    # riptide/tests/test_ffa_base_functions.py:35-56 (rotation + zero padding invariance)
    for shift in range(8):
        x = np.roll(inputs.FFA_IN_88, shift, axis=1)
        assert np.array_equal(oracle.ffa2(x), np.roll(inputs.FFA_OUT_88, shift, axis=1))
    for extra in range(8):
        x = np.hstack([inputs.FFA_IN_88, np.zeros((8, extra), np.float32)])
        y = np.hstack([inputs.FFA_OUT_88, np.zeros((8, extra), np.float32)])
        assert np.array_equal(oracle.ffa2(x), y)
    assert np.array_equal(golden["ffa2_88_out"], inputs.FFA_OUT_88)


@pytest.mark.parametrize("m,p,seed", inputs.FFA_CASES)
@pytest.mark.parametrize("fma", [0, 1])
def test_ffa2_bit_exact(oracle, golden, m, p, seed, fma):
    """Both index forms (fused and unfused kh*s+0.5f) reproduce the reference."""
    oracle.lib().oracle_set_index_fma(fma)
    try:
        y = oracle.ffa2(inputs.ffa_block(m, p, seed))
    finally:
        oracle.lib().oracle_set_index_fma(1)
    assert sha(y) == str(golden[f"ffa2_{m}x{p}_sha"])


@pytest.mark.parametrize("f", inputs.DS_FACTORS)
def test_downsample(oracle, golden, f):
    x = inputs.noise(20000, 11)
    ref = golden[f"downsample_{f!r}"]
    out = oracle.downsample(x, f)
    assert out.shape == ref.shape
    # float32 summation order differs from the -ffast-math build (vectorised sum)
    assert np.allclose(out, ref, rtol=2e-6, atol=2e-5 * max(1.0, f ** 0.5))


def test_snr2_and_prefix(oracle, golden):
    prof = inputs.noise(200 * 250, 12).reshape(200, 250)
    prof[:, 100:113] += 3.0
    ok, msg = snr_close(oracle.snr2(prof, inputs.SNR_WIDTHS, 1.7), golden["snr2_out"])
    assert ok, msg
    cps = oracle.circular_prefix_sum(prof[0], 700)
    assert np.allclose(cps, golden["cps_out"], rtol=1e-6, atol=1e-5)


@pytest.mark.parametrize("w", inputs.RMED_WIDTHS)
def test_running_median_exact(oracle, golden, w):
    x = inputs.noise(1000, 13)
    assert np.array_equal(oracle.running_median(x, w), golden[f"rmed_{w}"])


@pytest.mark.parametrize("ws,mp", inputs.FAST_RMED_CASES)
def test_fast_running_median(oracle, golden, ws, mp):
    x = inputs.noise(30011, 14)
    out = oracle.fast_running_median(x, ws, mp)
    assert np.array_equal(out, golden[f"frmed_{ws}_{mp}"])


@pytest.mark.parametrize("case", inputs.PGRAM_CASES, ids=lambda c: c["name"])
def test_periodogram(oracle, golden, case):
    name = case["name"]
    data = inputs.pgram_input(case)
    assert sha(data) == str(golden[f"pg_{name}_input_sha"])
    widths = oracle.generate_width_trials(case["bmin"], case["ducy_max"])
    assert np.array_equal(widths, golden[f"pg_{name}_widths"])
    periods, foldbins, snrs = oracle.periodogram(data, case["tsamp"], widths, case["pmin"],
                                                 case["pmax"], case["bmin"], case["bmax"])
    assert np.array_equal(periods, golden[f"pg_{name}_periods"])  # bit-exact grid
    assert np.array_equal(foldbins, golden[f"pg_{name}_foldbins"])
    ok, msg = snr_close(snrs, golden[f"pg_{name}_snrs"])
    assert ok, msg


@pytest.mark.parametrize("name", ["cfg1", "cfg2", "cfg3", "cfg4"])
def test_full_grid_bit_exact(oracle, golden_full, name):
    """Full-size BASELINE configs: the grid (periods, foldbins, L) is bit-exact."""
    g = golden_full["configs"][name]
    c = g["case"]
    widths = oracle.generate_width_trials(c["bmin"], c["ducy_max"])
    assert [int(w) for w in widths] == g["widths"]
    L = oracle.periodogram_length(c["n"], c["tsamp"], c["pmin"], c["pmax"], c["bmin"], c["bmax"])
    assert L == g["length"]
    periods, foldbins, _ = oracle.periodogram(np.zeros(c["n"], np.float32), c["tsamp"], widths,
                                              c["pmin"], c["pmax"], c["bmin"], c["bmax"], grid_only=True)
    assert sha(periods) == g["periods_sha"]
    assert sha(foldbins) == g["foldbins_sha"]


def test_grid_source_form_differs(oracle, golden):
    """Documents SURVEY.md §0 finding 2: the source-text grid expression is NOT
    what the reference binary computes; the emitted fma form is."""
    case = inputs.PGRAM_CASES[0]
    widths = oracle.generate_width_trials(case["bmin"], case["ducy_max"])
    oracle.lib().oracle_set_grid_emitted(0)
    try:
        periods, _, _ = oracle.periodogram(np.zeros(case["n"], np.float32), case["tsamp"], widths,
                                           case["pmin"], case["pmax"], case["bmin"], case["bmax"], grid_only=True)
    finally:
        oracle.lib().oracle_set_grid_emitted(1)
    assert not np.array_equal(periods, golden["pg_cfg1_periods"])
    assert np.allclose(periods, golden["pg_cfg1_periods"], rtol=1e-15, atol=0)


@pytest.mark.parametrize("case", inputs.SEARCH_CASES, ids=lambda c: c["name"])
def test_search_pipeline(oracle, golden, case):
    """deredden + normalise + periodogram restated in numpy vs the reference."""
    name = case["name"]
    raw = inputs.search_input(case)
    assert sha(raw) == str(golden[f"search_{name}_input_sha"])
    x, widths, periods, foldbins, snrs = oracle.ffa_search_arrays(
        raw, case["tsamp"], case["pmin"], case["pmax"], case["bmin"], case["bmax"],
        ducy_max=case["ducy_max"], rmed_width=case["rmed_width"], rmed_minpts=case["rmed_minpts"])
    assert sha(x) == str(golden[f"search_{name}_normalised_sha"])
    assert sha(periods) == str(golden[f"search_{name}_periods_sha"])
    ok, msg = snr_close(snrs, golden[f"search_{name}_snrs"])
    assert ok, msg


# ---------------------------------------------------------------- input generators (CPU)
# The full-size GPU parity tests regenerate their inputs on the box and fail
# (not skip) when a generator drifts; these pin the same sha256s on the CPU, so
# a numpy/libm change shows up in the CPU suite first.
@pytest.mark.parametrize("name", ["cfg1", "cfg2", "cfg3", "cfg4"])
def test_full_input_generators_pinned(golden_full, name):
    g = golden_full["configs"][name]
    assert sha(inputs.full_input(g["case"])) == g["input_sha"]


def test_cfg5_input_generator_pinned():
    import json
    import os
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden_e2e.json")) as f:
        e2e = json.load(f)
    for f in e2e["cfg5"]["files"][:3]:
        data, _ = inputs.cfg5_trial(f["k"])
        assert sha(data) == f["input_sha"], f"cfg5 trial {f['k']}"
