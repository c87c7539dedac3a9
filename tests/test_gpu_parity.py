"""Parity of the HIP path (through the C ABI) with the oracle and the golden
vectors of the reference.  Bit-exact: FFA transform, downsample (vs the strict
oracle), trial grid, running median, dereddened series.  S/N: 1e-4 relative
(BASELINE.json), scaled by max(|ref|, 1) since S/N is in units of sigma.
"""
import hashlib
import os

import numpy as np
import pytest

import inputs
from conftest import snr_close

pytestmark = pytest.mark.gpu


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.fixture(scope="module")
def rt():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")
    import riptide_amd
    return riptide_amd


# ---------------------------------------------------------------- FFA transform
def test_ffa_known_answer(rt):
    # test_ffa_base_functions.py:35-56
    for shift in range(8):
        x = np.roll(inputs.FFA_IN_88, shift, axis=1)
        truth = np.roll(inputs.FFA_OUT_88, shift, axis=1)
        assert np.array_equal(rt.ffa2(x), truth)
        assert np.array_equal(rt.ffa1(x.ravel(), 8), truth)
    for extra in range(8):
        x = np.hstack([inputs.FFA_IN_88, np.zeros((8, extra))])
        truth = np.hstack([inputs.FFA_OUT_88, np.zeros((8, extra))])
        assert np.array_equal(rt.ffa2(x), truth)


@pytest.mark.parametrize("m,p,seed", inputs.FFA_CASES)
def test_ffa2_golden_bit_exact(rt, golden, m, p, seed):
    y = rt.ffa2(inputs.ffa_block(m, p, seed))
    assert y.shape == (m, p) and y.dtype == np.float32
    assert sha(y) == str(golden[f"ffa2_{m}x{p}_sha"])


@pytest.mark.parametrize("m,p", [(1, 1), (2, 1), (7, 3), (33, 64), (150, 260), (1023, 34), (1025, 34),
                                 (5000, 260), (21474, 240), (134217, 16), (3000, 17), (777, 4000),
                                 (40, 12000), (9, 70000),
                                 # short rows: every interleaved-task segment count (p = 9-32) with p
                                 # a multiple of 8 and not (bins past p land in the row padding)
                                 (999, 9), (1500, 12), (5000, 20), (4099, 24), (2049, 27), (3001, 31),
                                 (65537, 32),
                                 # 5-slot rows: through the roll table (257-260 bins: one and four
                                 # fifth-slot bins) and without it (261-320)
                                 (3001, 257), (2999, 260), (4099, 261), (2000, 300), (1000, 320),
                                 # wide rows, every slot-width variant and its edges (8: 321-512,
                                 # 11: 513-704, 16: 705-1024, 22: 1025-1408, 45: 1409-2880)
                                 (3000, 512), (3001, 513), (2500, 520), (1999, 704), (1500, 705),
                                 (1201, 1024), (1201, 1025), (1100, 1040), (900, 1408), (700, 1409),
                                 (333, 2880)])
def test_ffa2_vs_oracle(rt, oracle, m, p):
    x = np.random.RandomState(m * 31 + p).normal(size=(m, p)).astype(np.float32)
    assert np.array_equal(rt.ffa2(x), oracle.ffa2(x))


def test_ffa2_edge_and_errors(rt):
    assert rt.ffa2(np.zeros((0, 5), np.float32)).shape == (0, 5)
    with pytest.raises(ValueError):
        rt.ffa2(np.zeros(4))
    with pytest.raises(ValueError):
        rt.ffa1(np.zeros((4, 4)), 4)
    with pytest.raises(ValueError):
        rt.ffa1(np.zeros(10), 11)
    with pytest.raises(ValueError):
        rt.ffa1(np.zeros(10), 4.0)
    with pytest.raises(ValueError):
        rt.ffa2(np.zeros((16, 8), np.float32)[:, ::2])   # non-contiguous float32


# ---------------------------------------------------------------- downsample
@pytest.mark.parametrize("f", inputs.DS_FACTORS)
def test_downsample(rt, oracle, golden, f):
    x = inputs.noise(20000, 11)
    out = rt.downsample(x, f)
    assert np.array_equal(out, oracle.downsample(x, f))          # strict restatement: bit-exact
    assert np.allclose(out, golden[f"downsample_{f!r}"], rtol=2e-6, atol=2e-5 * max(1.0, f ** 0.5))


def test_downsample_errors(rt):
    x = np.zeros(100, np.float32)
    for f in (0.55, 1.0, 101.0):
        with pytest.raises(ValueError):
            rt.downsample(x, f)


# ---------------------------------------------------------------- S/N
def test_snr2_golden(rt, oracle, golden):
    prof = inputs.noise(200 * 250, 12).reshape(200, 250)
    prof[:, 100:113] += 3.0
    out = rt.boxcar_snr(prof, inputs.SNR_WIDTHS, 1.7)
    ok, msg = snr_close(out, golden["snr2_out"])
    assert ok, msg
    ok, msg = snr_close(out, oracle.snr2(prof, inputs.SNR_WIDTHS, 1.7), rtol=2e-6)
    assert ok, msg


def test_snr_reference_cases(rt):
    # test_snr.py:7-78
    data = np.zeros(32, np.float32)
    for bad in ([0, 1], [1, 32]):
        with pytest.raises(ValueError):
            rt.boxcar_snr(data, bad)
    with pytest.raises(ValueError):
        rt.boxcar_snr(data, [1, 2], stdnoise=-42.0)
    assert rt.boxcar_snr(np.zeros((3, 4, 32), np.float32), [1, 2, 3, 5]).shape == (3, 4, 4)
    rows = np.random.RandomState(0).normal(size=(4, 32)).astype(np.float32)
    ref = rt.boxcar_snr(rows, [1, 2, 5, 11, 18, 31])
    for shift in range(1, 33):
        assert np.allclose(rt.boxcar_snr(np.roll(rows, shift, axis=-1), [1, 2, 5, 11, 18, 31]), ref)
    n = 64
    widths = np.arange(1, n)
    d = np.zeros(n, np.float32)
    for w in range(1, n):
        d[:w] = 1.0
        s = rt.boxcar_snr(d, widths)
        assert s.argmax() == w - 1
        assert np.allclose(s.max(), w * np.sqrt((n - w) / (n * w)))


def test_circular_prefix_sum_and_rollback(rt, golden):
    from riptide_amd import libcpp
    prof = inputs.noise(200 * 250, 12).reshape(200, 250)
    prof[:, 100:113] += 3.0
    assert np.allclose(libcpp.circular_prefix_sum(prof[0].copy(), 700), golden["cps_out"], rtol=1e-6, atol=1e-5)
    x = np.arange(10, dtype=np.float32)
    y = np.arange(10, dtype=np.float32) * 10
    for s in (0, 3, 10, 13):
        assert np.array_equal(libcpp.rollback(x, s), np.roll(x, -s))
        assert np.array_equal(libcpp.fused_rollback_add(x, y, s), x + np.roll(y, -s))
    with pytest.raises(ValueError):
        libcpp.fused_rollback_add(x, y[:5], 1)


# ---------------------------------------------------------------- running median
@pytest.mark.parametrize("w", inputs.RMED_WIDTHS)
def test_running_median_exact(rt, golden, w):
    assert np.array_equal(rt.running_median(inputs.noise(1000, 13), w), golden[f"rmed_{w}"])


def test_running_median_reference_cases(rt):
    # test_running_median.py:16-73
    data = np.arange(10, dtype=np.float32)
    for args in ((data, 2), (data, 10), (np.zeros((4, 8)), 3)):
        with pytest.raises(ValueError):
            rt.running_median(*args)
    rs = np.random.RandomState(5)
    x = rs.normal(size=300).reshape(100, 3).astype(np.float32)
    for col in x.T:                 # non-contiguous slices
        for w in (1, 3, 5, 7, 11, 25, 37):
            padded = np.pad(col, (w // 2, w // 2), mode="edge")
            naive = np.array([np.median(padded[i:i + w]) for i in range(col.size)])
            assert np.array_equal(rt.running_median(col, w), naive)
    with pytest.raises(ValueError):
        rt.fast_running_median(np.zeros(100), 3, min_points=10)
    x64 = rs.normal(size=100)
    for w in (1, 3, 5, 7, 11, 25, 37):
        assert np.array_equal(rt.running_median(x64, w), rt.fast_running_median(x64, w, min_points=39))


@pytest.mark.parametrize("run", ["3", "5", "7", "9"])
def test_running_median_walk_matches_counting(rt, monkeypatch, run):
    """The run kernel's walk in sorted order (rmed_run_kernel<RUN>, every
    instantiation: RIPTIDE_AMD_RMED_RUN is read per launch) returns the
    same element as the full counting search (rmed_small_kernel,
    RIPTIDE_AMD_RMED_COUNTING=1), bit for bit (the sign of zero included), on
    data that defeats its near-median start or its walk: heavy duplicates,
    +0.0 / -0.0 mixes, monotone runs, step changes, outliers, infinities and
    NaNs."""
    monkeypatch.setenv("RIPTIDE_AMD_RMED_RUN", run)
    rs = np.random.RandomState(11)
    n = 5003
    cases = [np.round(rs.normal(size=n) * 2.0) / 2.0,                        # few distinct values
             np.where(rs.rand(n) < 0.5, 0.0, -0.0) + np.where(rs.rand(n) < 0.1, rs.normal(size=n), 0.0),
             np.arange(n, dtype=np.float64), np.arange(n, 0, -1, dtype=np.float64),
             np.where(np.arange(n) % 400 < 200, 100.0, -100.0) + rs.normal(size=n),
             rs.standard_cauchy(size=n),
             np.where(rs.rand(n) < 0.02, np.inf, rs.normal(size=n)),
             np.where(rs.rand(n) < 0.02, -np.inf, rs.normal(size=n)),
             np.where(rs.rand(n) < 0.05, np.nan, rs.normal(size=n))]
    for w in (3, 37, 101, 255):
        for x in cases:
            x = x.astype(np.float32)
            monkeypatch.setenv("RIPTIDE_AMD_RMED_COUNTING", "1")
            ref = rt.running_median(x, w)
            monkeypatch.delenv("RIPTIDE_AMD_RMED_COUNTING")
            got = rt.running_median(x, w)
            assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), w


@pytest.mark.parametrize("ws", [203, 303, 404, 1001, 15625])
def test_deredden_normalise_batch_vs_oracle(rt, oracle, monkeypatch, ws):
    """Device dereddening of a batch (scrunch factors 2, 3, 4, 9, 154: the
    two-segment fast interpolation needs factor >= 4, the others take the
    per-sample form) bit-identical to the oracle's fast_running_median
    subtraction, and the normalisation -- statistics summed by the
    dereddening kernel, or by their own read passes with
    RIPTIDE_AMD_NORM_UNFUSED -- within 2e-6 of the oracle's numpy
    mean / var.  Rows of 30011 samples in 16-byte aligned rows of 30016
    floats: the 16-byte path with a ragged last group."""
    import torch
    from riptide_amd import engine
    n, B, mp = 30011, 3, 101
    rs = np.random.RandomState(ws)
    xs = (rs.normal(size=(B, n)) + 5.0 + np.sin(np.arange(n) / 700.0)).astype(np.float32)
    big = torch.zeros((B, 30016), dtype=torch.float32, device="cuda")
    big[:, :n] = torch.from_numpy(xs).cuda()
    x = big[:, :n]
    dered = engine.deredden_normalise(x, ws, mp, normalise=False).cpu().numpy()        # one-sample form
    ob = torch.zeros((B, 30016), dtype=torch.float32, device="cuda")
    engine.deredden_normalise(x, ws, mp, normalise=False, out=ob[:, :n])
    dered4 = ob[:, :n].cpu().numpy()                                                       # 16-byte form
    outs = {}
    for unfused in (False, True):
        if unfused:
            monkeypatch.setenv("RIPTIDE_AMD_NORM_UNFUSED", "1")
        else:
            monkeypatch.delenv("RIPTIDE_AMD_NORM_UNFUSED", raising=False)
        ob = torch.zeros((B, 30016), dtype=torch.float32, device="cuda")
        engine.deredden_normalise(x, ws, mp, out=ob[:, :n])
        outs[unfused] = ob[:, :n].cpu().numpy()
    for b in range(B):
        ref = np.asarray(xs[b] - oracle.fast_running_median(xs[b], ws, mp), dtype=np.float32)
        assert np.array_equal(dered[b], ref) and np.array_equal(dered4[b], ref)
        norm = oracle.normalise(ref)
        for unfused in (False, True):
            assert np.allclose(outs[unfused][b], norm, rtol=2e-6, atol=2e-6)
        # the fused statistics (one-pass E[x^2] - m^2, summed in the
        # dereddening kernel: 16-byte aligned rows) and the two-pass ones
        # (unaligned buffers, or RIPTIDE_AMD_NORM_UNFUSED) may differ in the
        # last bits; the bound DESIGN.md §3.3 states: <= 2e-6 x max(|x|, 1)
        d = np.abs(outs[False][b].astype(np.float64) - outs[True][b])
        assert np.all(d <= 2e-6 * np.maximum(np.abs(norm), 1.0)), float(d.max())


@pytest.mark.parametrize("ws,mp", inputs.FAST_RMED_CASES)
def test_fast_running_median_exact(rt, golden, ws, mp):
    out = rt.fast_running_median(inputs.noise(30011, 14), ws, mp)
    assert np.array_equal(out, golden[f"frmed_{ws}_{mp}"])


# ---------------------------------------------------------------- periodogram
@pytest.mark.parametrize("case", inputs.PGRAM_CASES, ids=lambda c: c["name"])
def test_periodogram_golden(rt, oracle, golden, case):
    from riptide_amd import libcpp
    name = case["name"]
    data = inputs.pgram_input(case)
    widths = golden[f"pg_{name}_widths"]
    periods, foldbins, snrs = libcpp.periodogram(data, case["tsamp"], widths, case["pmin"], case["pmax"],
                                                 case["bmin"], case["bmax"])
    assert np.array_equal(periods, golden[f"pg_{name}_periods"])
    assert np.array_equal(foldbins, golden[f"pg_{name}_foldbins"])
    ok, msg = snr_close(snrs, golden[f"pg_{name}_snrs"])
    assert ok, msg
    _, _, osnrs = oracle.periodogram(data, case["tsamp"], widths, case["pmin"], case["pmax"],
                                     case["bmin"], case["bmax"])
    ok, msg = snr_close(snrs, osnrs, rtol=2e-6)
    assert ok, msg


@pytest.mark.parametrize("case", inputs.SEARCH_CASES, ids=lambda c: c["name"])
def test_ffa_search_pipeline(rt, golden, case):
    name = case["name"]
    raw = inputs.search_input(case)
    ts = rt.TimeSeries(raw, case["tsamp"])
    tsdr, pg = rt.ffa_search(ts, period_min=case["pmin"], period_max=case["pmax"], bins_min=case["bmin"],
                             bins_max=case["bmax"], ducy_max=case["ducy_max"], rmed_width=case["rmed_width"],
                             rmed_minpts=case["rmed_minpts"])
    head = golden[f"search_{name}_normalised_head"]
    assert np.allclose(tsdr.data[:head.size], head, rtol=0, atol=2e-6)
    assert sha(pg.periods) == str(golden[f"search_{name}_periods_sha"])
    ok, msg = snr_close(pg.snrs, golden[f"search_{name}_snrs"])
    assert ok, msg
    pg.metadata["dm"] = 0.0
    peaks, _ = rt.find_peaks(pg)
    ref = golden[f"search_{name}_peaks"]
    got = np.array([(p.ip, p.iw, p.snr) for p in peaks], dtype=np.float64).reshape(-1, 3)
    assert got.shape == ref.shape
    assert np.array_equal(got[:, :2], ref[:, :2])           # identical candidate list
    assert np.allclose(got[:, 2], ref[:, 2], rtol=1e-4, atol=1e-4)


def test_ffa_search_reference_invariants(rt):
    # test_ffa_search_pgram.py:11-96
    np.random.seed(0)
    ts = rt.TimeSeries.generate(200.0, 0.001, 1.0, amplitude=20.0)
    tsdr, pg = rt.ffa_search(ts, period_min=0.8, period_max=1.2, bins_min=240, bins_max=260)
    assert np.all(np.maximum.accumulate(pg.periods) == pg.periods)
    assert pg.snrs.shape == (len(pg.periods), len(pg.widths))
    assert pg.metadata == ts.metadata == tsdr.metadata
    assert pg.tobs == 200.0
    assert np.all(pg.freqs == 1.0 / pg.periods)
    tsdr, pg = rt.ffa_search(ts, period_min=0.8, period_max=1.2, bins_min=240, bins_max=260,
                             already_normalised=True, deredden=False)
    assert id(tsdr) == id(ts)
    # no downsampling: period_min = bins_min * tsamp (f == 1 rung)
    rt.ffa_search(ts, period_min=0.8, period_max=1.2, bins_min=800, bins_max=1200)


def test_periodogram_errors(rt):
    from riptide_amd import libcpp
    x = np.zeros(10000, np.float32)
    w = np.array([1, 2], dtype=np.uint64)
    bad = [(0.0, 1.0, 2.0), (1e-3, 0.0, 2.0), (1e-3, 1.0, 0.5), (1e-3, 0.01, 2.0)]
    for tsamp, pmin, pmax in bad:
        with pytest.raises(ValueError):
            libcpp.periodogram(x, tsamp, w, pmin, pmax, 240, 260)
    with pytest.raises(ValueError):
        libcpp.periodogram(x, 1e-3, w, 1.0, 2.0, 1, 260)
    with pytest.raises(ValueError):
        libcpp.periodogram(x, 1e-3, w, 1.0, 2.0, 240, 200)


# ---------------------------------------------------------------- device batch API
def test_batch_matches_single(rt):
    import torch
    from riptide_amd import engine
    case = inputs.PGRAM_CASES[1]
    plan = engine.PeriodogramPlan.for_search(case["n"], case["tsamp"], case["pmin"], case["pmax"],
                                             case["bmin"], case["bmax"], ducy_max=case["ducy_max"])
    xs = np.stack([inputs.with_signal(case["n"], case["tsamp"], s, 0.41, 12.0) for s in range(5)])
    d = torch.from_numpy(xs).cuda()
    batch = plan.run(d).cpu().numpy()
    from riptide_amd import libcpp
    for b in range(5):
        _, _, single = libcpp.periodogram(xs[b], case["tsamp"], plan.widths, case["pmin"], case["pmax"],
                                          case["bmin"], case["bmax"])
        assert np.array_equal(batch[b], single)
    dn = engine.deredden_normalise(d, 1001, 101)
    for b in range(2):
        ref = libcpp.deredden_normalise(xs[b], 1001, 101)
        assert np.array_equal(dn[b].cpu().numpy(), ref)


@pytest.mark.parametrize("tpw", ["1", "2", "3", "16"])
@pytest.mark.parametrize("ci", [0, 1, 3, 4])
def test_trials_per_workgroup(rt, monkeypatch, tpw, ci):
    """Workgroups running several trials of an item (RIPTIDE_AMD_TRIALS_PER_WG,
    ConeArgs::trials_per_wg; 16 by default): a batch of 5 distinct trials --
    T = 2 and 3 leave a partial last group -- bit-identical to each trial run
    alone, for the 4/5-slot rows (cfg2 / cfg1 search parameters) and the
    short rows (cfg4) and the 16-slot rows (800-1200 bins)."""
    import torch
    from riptide_amd import engine
    case = inputs.PGRAM_CASES[ci]
    monkeypatch.setenv("RIPTIDE_AMD_TRIALS_PER_WG", tpw)
    plan = engine.PeriodogramPlan.for_search(case["n"], case["tsamp"], case["pmin"], case["pmax"],
                                             case["bmin"], case["bmax"], ducy_max=case["ducy_max"])
    xs = np.stack([inputs.with_signal(case["n"], case["tsamp"], s, case["period"], 12.0) for s in range(5)])
    d = torch.from_numpy(xs).cuda()
    batch = plan.run(d, check=True).cpu().numpy()
    for b in range(5):
        single = plan.run(d[b:b + 1].contiguous(), check=True).cpu().numpy()[0]
        assert np.array_equal(batch[b], single), f"trial {b} differs in a batch at {tpw} trials per workgroup"


@pytest.mark.parametrize("tpw", ["2", "16"])
def test_trials_per_workgroup_segmented_snr(rt, monkeypatch, tpw):
    """The trial loop over final units that run the segmented S/N:
    cfg2 search parameters at 2^19 samples (a multi-pass schedule whose final
    tiles of 240-260-bin rows, widths <= 9, take snr_segments), batch 5, 2 and
    16 trials per workgroup -- every trial bit-identical to its batch-1 run,
    so the zero-row rewrite and the next trial's fill after the S/N's maxima
    and exchange areas leave no cross-trial state."""
    import torch
    from riptide_amd import engine
    n, tsamp = 1 << 19, 256e-6
    monkeypatch.setenv("RIPTIDE_AMD_TRIALS_PER_WG", tpw)
    plan = engine.PeriodogramPlan.for_search(n, tsamp, 0.1, 10.0, 240, 260, ducy_max=0.05)
    assert max(int(w) for w in plan.widths) <= 9
    xs = np.stack([inputs.with_signal(n, tsamp, 40 + s, 0.37 + 0.2 * s, 10.0) for s in range(5)])
    d = torch.from_numpy(xs).cuda()
    batch = plan.run(d, check=True).cpu().numpy()
    for b in range(5):
        single = plan.run(d[b:b + 1].contiguous(), check=True).cpu().numpy()[0]
        assert np.array_equal(batch[b], single), f"trial {b} differs in a batch at {tpw} trials per workgroup"


def test_ladder_passes_pipeline_matches_run(rt):
    """rt_periodogram_ladder_device + rt_periodogram_passes_device (the two
    halves a pipelined caller runs on two streams, bench.py --overlap 1) give
    exactly rt_periodogram_device's S/N: two batches with the second batch's
    ladder on a side stream while the first batch's passes run, one
    workspace per batch in flight."""
    import torch
    from riptide_amd import engine
    case = inputs.PGRAM_CASES[1]
    plan = engine.PeriodogramPlan.for_search(case["n"], case["tsamp"], case["pmin"], case["pmax"],
                                             case["bmin"], case["bmax"], ducy_max=case["ducy_max"])
    xs = [np.stack([inputs.with_signal(case["n"], case["tsamp"], s + 3 * k, 0.41, 12.0) for s in range(3)])
          for k in range(2)]
    ds = [torch.from_numpy(x).cuda() for x in xs]
    ref = [plan.run(d).cpu().numpy() for d in ds]
    ws = [torch.empty(plan.workspace_bytes(3), dtype=torch.uint8, device="cuda") for _ in range(2)]
    outs = [torch.empty((3, plan.length, plan.num_widths), dtype=torch.float32, device="cuda") for _ in range(2)]
    main, side = torch.cuda.current_stream(), torch.cuda.Stream()
    ev = [torch.cuda.Event() for _ in range(2)]
    for k in range(2):
        with torch.cuda.stream(side):
            side.wait_stream(main)
            plan.ladder(ds[k], ws[k], stream=side)
            ev[k].record(side)
        main.wait_event(ev[k])
        plan.passes(outs[k], ws[k], stream=main)
    torch.cuda.synchronize()
    plan.check()
    for k in range(2):
        assert np.array_equal(outs[k].cpu().numpy(), ref[k])
    with pytest.raises(ValueError):
        plan.ladder(ds[0], torch.empty(16, dtype=torch.uint8, device="cuda"))


@pytest.mark.parametrize("ducy_max, widths", [(0.2, None), (0.35, [1, 2, 5, 13, 40, 77, 91])])
def test_wide_snr_matches_window_path(monkeypatch, ducy_max, widths):
    """Final units whose S/N reads the widths past its 12-column register
    window as plain LDS windows (the WIDE kernel instances, final tiles capped
    to the wide row stride) give exactly the S/N of the wrapped-window path
    (RIPTIDE_AMD_SNR_WIDE=0), which the golden tests pin to the oracle; on a
    cfg3-shaped multi-pass schedule, incl. widths up to 91 of 240 bins and
    unsorted widths."""
    import torch
    from riptide_amd import engine, libcpp
    n, tsamp = 1 << 19, 256e-6
    x = np.stack([inputs.with_signal(n, tsamp, s, 0.71, 9.0) for s in range(3)])
    d = torch.from_numpy(x).cuda()
    out = {}
    for v in ("1", "0"):
        monkeypatch.setenv("RIPTIDE_AMD_SNR_WIDE", v)
        if widths is None:
            plan = engine.PeriodogramPlan.for_search(n, tsamp, 0.2, 5.0, 240, 260, ducy_max=ducy_max)
        else:
            plan = engine.PeriodogramPlan(n, tsamp, list(reversed(widths)), 0.2, 5.0, 240, 260)
        out[v] = plan.run(d).cpu().numpy()
    assert np.array_equal(out["1"], out["0"])
    w = [int(v) for v in plan.widths]
    _, _, single = libcpp.periodogram(x[1], tsamp, np.asarray(w, dtype=np.uint64), 0.2, 5.0, 240, 260)
    assert np.array_equal(out["1"][1], single)


@pytest.mark.parametrize("widths, bins", [(0.05, (240, 260)), (0.2, (240, 260)), ([9, 3, 1], (240, 265)),
                                          ([1, 5, 7, 8], (240, 265)), ([2], (250, 265)),
                                          ([120, 1, 2, 5, 13, 40, 77, 91, 215], (240, 265)),
                                          ([10, 11, 12, 13, 14, 15, 16, 17, 18, 2], (240, 262))])
def test_segmented_snr_matches_window_path(oracle, monkeypatch, widths, bins):
    """Final units of 240-264-bin rows with widths <= 9 run the segmented S/N
    (one row per lane, 8 column segments, rows in 265-float slots; plans with
    a wider width keep the window path, measured faster for them, r05y); it
    gives
    exactly the S/N of the wrapped-window path (feature bit kConeSnrSeg off:
    RIPTIDE_AMD_CONE_FLAGS=7) and of the single-trial run, and the strict C
    oracle's at test_full_config_every_row's tolerance, on a multi-pass schedule:
    the standard ladders of ducy_max 0.05 and 0.2, unsorted and non-ladder
    widths (5, 7, 8), a single width, widths up to 215, and rows of 240 bins
    (24 slack columns) up to 264 (none)."""
    import torch
    from riptide_amd import engine, libcpp
    n, tsamp = 1 << 19, 256e-6
    x = np.stack([inputs.with_signal(n, tsamp, s, 0.53, 7.0) for s in range(3)])
    d = torch.from_numpy(x).cuda()
    out = {}
    for v in ("15", "7"):
        monkeypatch.setenv("RIPTIDE_AMD_CONE_FLAGS", v)
        if isinstance(widths, float):
            plan = engine.PeriodogramPlan.for_search(n, tsamp, 0.2, 5.0, bins[0], bins[1], ducy_max=widths)
        else:
            plan = engine.PeriodogramPlan(n, tsamp, widths, 0.2, 5.0, bins[0], bins[1])
        out[v] = plan.run(d).cpu().numpy()
    monkeypatch.delenv("RIPTIDE_AMD_CONE_FLAGS")
    assert np.array_equal(out["15"], out["7"])
    w = [int(v) for v in plan.widths]
    _, _, single = libcpp.periodogram(x[2], tsamp, np.asarray(w, dtype=np.uint64), 0.2, 5.0, bins[0], bins[1])
    assert np.array_equal(out["15"][2], single)
    _, _, osnr = oracle.periodogram(x[2], tsamp, np.asarray(w, dtype=np.uint64), 0.2, 5.0, bins[0], bins[1],
                                    threads=min(16, os.cpu_count() or 1))
    ok, msg = snr_close(out["15"][2], osnr, rtol=2e-6)
    assert ok, msg


def test_fused_ladder_matches_per_rung(monkeypatch):
    """The fused downsampling ladder (one read of the series for every rung)
    produces exactly the per-rung kernel's leaves, hence identical S/N (odd batch:
    the two-trial blocks' last block holds one trial)."""
    import torch
    from riptide_amd import engine
    cases = [inputs.PGRAM_CASES[1], dict(n=1 << 22, tsamp=256e-6, pmin=0.1, pmax=10.0, bmin=240, bmax=260,
                                         ducy_max=0.05),
             inputs.LADDER_EDGE_CASE]        # largest rung at the fused kernel's margin
    for case in cases:
        x = torch.from_numpy(np.random.RandomState(7).normal(size=(3, case["n"])).astype(np.float32)).cuda()
        outs = []
        for per_rung in (False, True):
            if per_rung:
                monkeypatch.setenv("RIPTIDE_AMD_PER_RUNG_LADDER", "1")
            else:
                monkeypatch.delenv("RIPTIDE_AMD_PER_RUNG_LADDER", raising=False)
            plan = engine.PeriodogramPlan.for_search(case["n"], case["tsamp"], case["pmin"], case["pmax"],
                                                     case["bmin"], case["bmax"], ducy_max=case["ducy_max"])
            outs.append(plan.run(x).cpu().numpy())
        assert np.array_equal(outs[0], outs[1])


def test_fused_ladder_leaves_match_per_rung(monkeypatch):
    """The fused ladder's leaves themselves (every rung's downsampled series,
    the workspace's leaf buffer after plan.ladder) equal the per-rung kernel's
    bit for bit: cfg2's full-size 57-rung ladder, the margin edge case, a
    short odd-length series (the clipping tail block), cfg4, and cfg5's long
    range (factors 30-1950: the rungs past the margin in the per-rung kernel
    beside the fused one, rt_ladder_check = 2)."""
    import torch
    from riptide_amd import engine
    cases = [dict(n=1 << 23, tsamp=256e-6, pmin=0.1, pmax=10.0, bmin=240, bmax=260, ducy_max=0.2),
             inputs.LADDER_EDGE_CASE, dict(inputs.PGRAM_CASES[1], n=inputs.PGRAM_CASES[1]["n"] - 37),
             inputs.PGRAM_CASES[3],
             dict(n=1 << 21, tsamp=64e-6, pmin=2.0, pmax=120.0, bmin=960, bmax=1040, ducy_max=0.2)]
    for case in cases:
        x = torch.from_numpy(np.random.RandomState(11).normal(size=(2, case["n"])).astype(np.float32)).cuda()
        leaves = []
        for per_rung in (False, True):
            if per_rung:
                monkeypatch.setenv("RIPTIDE_AMD_PER_RUNG_LADDER", "1")
            else:
                monkeypatch.delenv("RIPTIDE_AMD_PER_RUNG_LADDER", raising=False)
            plan = engine.PeriodogramPlan.for_search(case["n"], case["tsamp"], case["pmin"], case["pmax"],
                                                     case["bmin"], case["bmax"], ducy_max=case["ducy_max"])
            ws = torch.zeros(plan.workspace_bytes(2), dtype=torch.uint8, device="cuda")
            plan.ladder(x, ws)
            torch.cuda.synchronize()
            leaves.append(ws)
        assert torch.equal(leaves[0], leaves[1]), case


# ---------------------------------------------------------------- full-size BASELINE configs
@pytest.mark.parametrize("name", ["cfg1", "cfg2", "cfg3", "cfg4"])
def test_full_config(rt, golden_full, name):
    import torch
    from riptide_amd import engine
    g = golden_full["configs"][name]
    c = g["case"]
    raw = inputs.full_input(c)
    if sha(raw) != g["input_sha"]:
        pytest.fail(f"input generator drifted on this host (numpy RNG/libm): input sha256 {sha(raw)} != golden "
                    f"{g['input_sha']}; the full-size parity check cannot run")
    plan = engine.PeriodogramPlan.for_search(c["n"], c["tsamp"], c["pmin"], c["pmax"], c["bmin"], c["bmax"],
                                             ducy_max=c["ducy_max"])
    assert [int(w) for w in plan.widths] == g["widths"] and plan.length == g["length"]
    periods, foldbins = plan.grid()
    assert sha(periods) == g["periods_sha"] and sha(foldbins) == g["foldbins_sha"]
    d = torch.from_numpy(raw).cuda()
    x = engine.deredden_normalise(d, int(round(4.0 / c["tsamp"])), 101)
    snrs = plan.run(x).cpu().numpy()
    _check_full_snrs(rt, g, c, plan, periods, foldbins, snrs)


def _check_full_snrs(rt, g, c, plan, periods, foldbins, snrs):
    """The golden_full checks of one full-size configuration's S/N."""
    # >= 5000 sampled rows, including the first and last evaluated row of
    # every FFA transform (tile / pass boundaries of the cone schedule)
    rows = np.asarray(g["sample_rows"])
    assert rows.size >= 5000 and set(g["boundary_rows"]) <= set(g["sample_rows"])
    ok, msg = snr_close(snrs[rows], np.asarray(g["sample_snrs"], dtype=np.float32))
    assert ok, msg
    assert np.allclose(snrs.max(axis=0), g["snr_max"], rtol=1e-4)
    assert list(snrs.argmax(axis=0)) == g["snr_argmax"]
    # every one of the L rows, per width, through its sum: |sum - ref| within
    # 1e-4 relative of sum |S/N| (each row's own bound, summed)
    s64 = snrs.astype(np.float64)
    assert np.all(np.abs(s64.sum(axis=0) - np.asarray(g["snr_sum"])) <= 1e-4 * np.asarray(g["snr_abs_sum"]))
    assert np.allclose(np.abs(s64).sum(axis=0), g["snr_abs_sum"], rtol=1e-5)
    pg = rt.Periodogram(plan.widths, periods, foldbins, snrs, metadata=rt.Metadata({"tobs": c["n"] * c["tsamp"],
                                                                                       "dm": 0.0}))
    peaks, _ = rt.find_peaks(pg)
    got = [[p.ip, p.iw] for p in peaks]
    assert got == [[p[0], p[1]] for p in g["peaks"]]     # identical candidate list


def test_bench_schedule_cfg2(rt, golden_full, monkeypatch):
    """The schedule bench.py times: the whole cfg2 plan
    in ONE transform group (RIPTIDE_AMD_SCRATCH_MFLOATS=1536: 14 cone
    launches, every transform's scratch side by side) at batch 2, against the
    golden cfg2 results (trial 0: the golden input) and bit-identical to the
    default 96 Mi-float grouping (both trials; trial 1 the golden input
    reversed, so the batch's trials differ)."""
    import torch
    from riptide_amd import engine
    g = golden_full["configs"]["cfg2"]
    c = g["case"]
    raw = inputs.full_input(c)
    if sha(raw) != g["input_sha"]:
        pytest.fail(f"input generator drifted on this host: input sha256 {sha(raw)} != golden {g['input_sha']}")
    args = (c["n"], c["tsamp"], c["pmin"], c["pmax"], c["bmin"], c["bmax"])
    monkeypatch.setenv("RIPTIDE_AMD_SCRATCH_MFLOATS", "1536")
    one = engine.PeriodogramPlan.for_search(*args, ducy_max=c["ducy_max"])
    monkeypatch.delenv("RIPTIDE_AMD_SCRATCH_MFLOATS")
    dflt = engine.PeriodogramPlan.for_search(*args, ducy_max=c["ducy_max"])
    s1, s0 = one.stats(), dflt.stats()
    assert s1["launches"] <= 16 < s0["launches"], (s1, s0)     # one group vs many
    d = torch.from_numpy(np.stack([raw, raw[::-1].copy()])).cuda()
    x = engine.deredden_normalise(d, int(round(4.0 / c["tsamp"])), 101)
    got = one.run(x, check=True)
    ref = dflt.run(x, check=True)
    torch.cuda.synchronize()
    assert torch.equal(got, ref), "one-group schedule differs from the default grouping"
    periods, foldbins = one.grid()
    _check_full_snrs(rt, g, c, one, periods, foldbins, got[0].cpu().numpy())


def _trial_variants(raw, B):
    """B distinct full-size series from the golden input:
    the input itself (trial 0), its reversal, sign flips and circular shifts
    -- same statistics, different S/N everywhere."""
    n = raw.size
    out = [raw, raw[::-1], -raw, -raw[::-1]]
    k = 1
    while len(out) < B:
        sh = np.roll(raw, (k * 1048573) % n)
        out.append(sh if k % 2 else -sh[::-1])
        k += 1
    return np.ascontiguousarray(np.stack(out[:B]))


@pytest.mark.parametrize("name,budget,cosched,batch", [("cfg2", "1024", True, 16), ("cfg2", "1536", False, 1),
                                                       ("cfg4", None, False, 16), ("cfg1", None, False, 1),
                                                       ("cfg3", "384", True, 32)])
def test_full_config_every_row(rt, oracle, golden_full, monkeypatch, name, budget, cosched, batch):
    """Every one of the L x W S/N values at full size (missing 3):
    the golden input through the schedule bench.py times for the config,
    compared element by element with the strict C oracle run on the same
    dereddened, normalised series (periodogram.hpp:175-194; threaded, same
    arithmetic per step) at the 2e-6 scaled tolerance of
    test_periodogram_golden, and with the golden sampled rows / sums / peaks
    of the reference build at 1e-4.  cfg2 at 1024 M co-scheduled is
    bench.py's schedule since round 5, at 1536 M its round-4 one.
    At the benchmarked batch (cfg2 / cfg4 16 trials, cfg3
    32 at 384 M co-scheduled) the golden input is trial 0 of a batch of
    distinct variants, so trials 1 .. B-1 of every workgroup run the trial
    loop's later-trial path (the next trial's fill over this trial's stores,
    the zero-row rewrite); each of them must equal its own batch-1 run through
    the same plan bit for bit, and trial 0 the oracle."""
    import torch
    from riptide_amd import engine
    g = golden_full["configs"][name]
    c = g["case"]
    raw = inputs.full_input(c)
    if sha(raw) != g["input_sha"]:
        pytest.fail(f"input generator drifted on this host: input sha256 {sha(raw)} != golden {g['input_sha']}")
    if budget:
        monkeypatch.setenv("RIPTIDE_AMD_SCRATCH_MFLOATS", budget)
    if cosched:
        monkeypatch.setenv("RIPTIDE_AMD_COSCHED", "1")
    args = (c["n"], c["tsamp"], c["pmin"], c["pmax"], c["bmin"], c["bmax"])
    plan = engine.PeriodogramPlan.for_search(*args, ducy_max=c["ducy_max"])
    if cosched and plan.workspace_bytes(batch) > 0.8 * torch.cuda.mem_get_info()[0]:
        # bench.py's own fallback when the second scratch bank does not fit
        monkeypatch.delenv("RIPTIDE_AMD_COSCHED")
        del plan
        plan = engine.PeriodogramPlan.for_search(*args, ducy_max=c["ducy_max"])
    d = torch.from_numpy(_trial_variants(raw, batch)).cuda()
    x = engine.deredden_normalise(d, int(round(4.0 / c["tsamp"])), 101)
    del d
    snr_dev = plan.run(x, check=True)
    torch.cuda.synchronize()
    if batch > 1:
        one = torch.empty((1, plan.length, plan.num_widths), dtype=torch.float32, device="cuda")
        ws = torch.empty(plan.workspace_bytes(1), dtype=torch.uint8, device="cuda")
        for b in range(batch):
            plan.run(x[b:b + 1], out=one, workspace=ws, check=True)
            torch.cuda.synchronize()
            nbad = int((one[0] != snr_dev[b]).sum().item())
            assert nbad == 0, f"{name}: trial {b} of the batch of {batch}: {nbad} S/N values differ from its batch-1 run"
        del one, ws
    snrs = snr_dev[0].cpu().numpy()
    del snr_dev
    periods, foldbins = plan.grid()
    op, ofb, osnr = oracle.periodogram(x[0].cpu().numpy(), c["tsamp"], np.asarray(plan.widths, dtype=np.uint64),
                                       c["pmin"], c["pmax"], c["bmin"], c["bmax"],
                                       threads=min(16, os.cpu_count() or 1))
    assert np.array_equal(periods, op) and np.array_equal(foldbins, ofb)
    assert osnr.shape == snrs.shape == (g["length"], len(g["widths"]))
    ok, msg = snr_close(snrs, osnr, rtol=2e-6)
    assert ok, f"{name}: all {snrs.size} S/N values vs the strict oracle: {msg}"
    _check_full_snrs(rt, g, c, plan, periods, foldbins, snrs)


def test_single_stream_matches_two_streams_cfg2(rt, golden_full, monkeypatch):
    """The two-stream slot-width chains (the default for plans with more than
    one slot width, capi.cpp run_cone_launches) against every launch on the
    caller's stream in plan order (RIPTIDE_AMD_SINGLE_STREAM=1): bit-identical
    S/N on the benchmarked cfg2 schedule, golden input and its reverse."""
    import torch
    from riptide_amd import engine
    g = golden_full["configs"]["cfg2"]
    c = g["case"]
    raw = inputs.full_input(c)
    monkeypatch.setenv("RIPTIDE_AMD_SCRATCH_MFLOATS", "1536")
    plan = engine.PeriodogramPlan.for_search(c["n"], c["tsamp"], c["pmin"], c["pmax"], c["bmin"], c["bmax"],
                                             ducy_max=c["ducy_max"])
    d = torch.from_numpy(np.stack([raw, raw[::-1].copy()])).cuda()
    x = engine.deredden_normalise(d, int(round(4.0 / c["tsamp"])), 101)
    two = plan.run(x, check=True)
    monkeypatch.setenv("RIPTIDE_AMD_SINGLE_STREAM", "1")
    one = plan.run(x, check=True)
    monkeypatch.delenv("RIPTIDE_AMD_SINGLE_STREAM")
    torch.cuda.synchronize()
    assert torch.equal(one, two), "single-stream schedule differs from the two-stream chains"


@pytest.mark.parametrize("budget", ["1024", "384", "96"])
def test_cosched_schedule_cfg2(rt, golden_full, monkeypatch, budget):
    """Co-scheduled transform groups (RIPTIDE_AMD_COSCHED=1: two scratch
    banks, group g on stream g mod 2, its merge-only launches overlapping
    group g - 1's final ones) give S/N bit-identical to the one-stream
    schedule, on the golden cfg2 input and its reverse (batch 2)."""
    import torch
    from riptide_amd import engine
    g = golden_full["configs"]["cfg2"]
    c = g["case"]
    raw = inputs.full_input(c)
    args = (c["n"], c["tsamp"], c["pmin"], c["pmax"], c["bmin"], c["bmax"])
    monkeypatch.setenv("RIPTIDE_AMD_SCRATCH_MFLOATS", budget)
    monkeypatch.setenv("RIPTIDE_AMD_COSCHED", "1")
    co = engine.PeriodogramPlan.for_search(*args, ducy_max=c["ducy_max"])
    monkeypatch.delenv("RIPTIDE_AMD_COSCHED")
    monkeypatch.delenv("RIPTIDE_AMD_SCRATCH_MFLOATS")
    ref = engine.PeriodogramPlan.for_search(*args, ducy_max=c["ducy_max"])
    d = torch.from_numpy(np.stack([raw, raw[::-1].copy()])).cuda()
    x = engine.deredden_normalise(d, int(round(4.0 / c["tsamp"])), 101)
    for _ in range(2):                      # the second run reuses the plan's side stream
        got = co.run(x, check=True)
        want = ref.run(x, check=True)
        torch.cuda.synchronize()
        assert torch.equal(got, want), "co-scheduled groups differ from the one-stream schedule"
    periods, foldbins = co.grid()
    _check_full_snrs(rt, g, c, co, periods, foldbins, got[0].cpu().numpy())


# ---------------------------------------------------------------- device peak detection
def _device_vs_host_peaks(rt, plan, snr_dev, tobs, dm=0.0, **kw):
    from riptide_amd.peaks import PeakFinder
    finder = PeakFinder(plan, tobs, **kw)
    dev = finder(snr_dev, dms=[dm] * snr_dev.shape[0])
    periods, foldbins = plan.grid()
    snrs = snr_dev.cpu().numpy()
    for b in range(snrs.shape[0]):
        pg = rt.Periodogram(plan.widths, periods, foldbins, snrs[b], metadata=rt.Metadata({"tobs": tobs, "dm": dm}))
        ref_peaks, ref_polycos = rt.find_peaks(pg, **kw)
        got_peaks, got_polycos = dev[b]
        assert got_peaks == ref_peaks                      # identical Peak tuples, same order
        for iw in ref_polycos:
            assert np.array_equal(np.asarray(got_polycos[iw]), np.asarray(ref_polycos[iw]))
    return dev


def test_device_find_peaks_matches_host(rt):
    import torch
    from riptide_amd import engine
    case = inputs.PGRAM_CASES[1]
    plan = engine.PeriodogramPlan.for_search(case["n"], case["tsamp"], case["pmin"], case["pmax"],
                                             case["bmin"], case["bmax"], ducy_max=case["ducy_max"])
    xs = np.stack([inputs.with_signal(case["n"], case["tsamp"], s, 0.41, 14.0) for s in range(4)])
    d = engine.deredden_normalise(torch.from_numpy(xs).cuda(), 1001, 101)
    snr = plan.run(d)
    tobs = case["n"] * case["tsamp"]
    dev = _device_vs_host_peaks(rt, plan, snr, tobs)
    assert any(len(p) for p, _ in dev)
    # a few threshold settings, including the constant-threshold branch (minseg)
    _device_vs_host_peaks(rt, plan, snr, tobs, smin=5.0, nstd=4.0)
    _device_vs_host_peaks(rt, plan, snr, tobs, minseg=10 ** 6)


@pytest.mark.parametrize("per_seg", [4097, 10000, 32768])
def test_segment_order_stats_long_segments(rt, per_seg):
    """Segments longer than 4096 points (the 1024-thread, dynamic-LDS sort;
    cfg5's short range has ~8K-point segments): the requested ranks of every
    (trial, width, segment) equal numpy's sorted values, NaN segments NaN."""
    import ctypes
    import torch
    from riptide_amd import _lib
    L_ = _lib.load()
    B, W, nseg = 2, 3, 3
    L = nseg * per_seg + 5
    rng = np.random.default_rng(per_seg)
    snr = rng.standard_normal((B, L, W)).astype(np.float32)
    snr[1, per_seg + 7, 2] = np.nan                     # trial 1, width 2, segment 1
    ranks = np.array([0, per_seg // 4, per_seg // 2, per_seg - 1], dtype=np.uint32)
    d = torch.from_numpy(snr).cuda()
    out = torch.empty((B, W, nseg, ranks.size), dtype=torch.float32, device="cuda")
    rc = L_.rt_segment_order_stats_device(_lib.ptr(d), B, L * W, L, W, nseg, per_seg, _lib.ptr(ranks), ranks.size,
                                          _lib.ptr(out), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0, L_.rt_last_error()
    got = out.cpu().numpy()
    for b in range(B):
        for iw in range(W):
            for sg in range(nseg):
                col = snr[b, sg * per_seg:(sg + 1) * per_seg, iw]
                if np.isnan(col).any():
                    assert np.isnan(got[b, iw, sg]).all()
                else:
                    assert np.array_equal(got[b, iw, sg], np.sort(col)[ranks])


@pytest.mark.parametrize("kind", ["rounded", "ties", "outlier", "inf", "zeros", "constant", "two_values", "tiny"])
def test_segment_order_stats_select_edge_cases(rt, kind):
    """The binned selection of segment_order_stats_kernel and its bitonic
    fallback on the distributions that stress them: heavy ties (small
    integers), a far outlier crowding the rest into one bin, +-inf values,
    signed zeros, constant and two-valued segments, values rounded to two
    decimals (ties inside the selected bins), and segments too short
    to bin -- the requested ranks (numpy's 'linear' percentile ranks and the
    extremes) equal numpy's sorted values."""
    import ctypes
    import torch
    from riptide_amd import _lib
    from riptide_amd.peaks import percentile_ranks
    L_ = _lib.load()
    rng = np.random.default_rng(7)
    for per_seg in ((1, 2, 3, 5, 64, 65) if kind == "tiny" else (97, 4096, 5000, 20000)):
        B, W, nseg = 2, 3, 2
        L = nseg * per_seg + 3
        if kind == "rounded":        # ties within the selected bins (binned path)
            snr = np.round(rng.standard_normal((B, L, W)), 2).astype(np.float32)
        elif kind == "ties":
            snr = rng.integers(-3, 4, (B, L, W)).astype(np.float32)
        elif kind == "outlier":
            snr = rng.standard_normal((B, L, W)).astype(np.float32)
            snr[:, ::max(per_seg // 3, 1), :] = 3.0e37
            snr[0, 1, 0] = -2.5e38
        elif kind == "inf":
            snr = rng.standard_normal((B, L, W)).astype(np.float32)
            snr[0, 2, :] = np.inf
            snr[1, per_seg + 1, :] = -np.inf
        elif kind == "zeros":
            snr = np.where(rng.random((B, L, W)) < 0.5, np.float32(-0.0), np.float32(0.0))
            snr[:, ::7, :] = rng.standard_normal((B, (L + 6) // 7, W))
        elif kind == "constant":
            snr = np.full((B, L, W), 4.25, dtype=np.float32)
        elif kind == "two_values":
            snr = np.where(rng.random((B, L, W)) < 0.3, np.float32(1.0), np.float32(1.0000001))
        else:
            snr = rng.standard_normal((B, L, W)).astype(np.float32)
        snr = np.ascontiguousarray(snr, dtype=np.float32)
        lohi, _ = percentile_ranks(per_seg)
        ranks = np.concatenate([lohi, [0, per_seg - 1]]).astype(np.uint32)
        d = torch.from_numpy(snr).cuda()
        out = torch.empty((B, W, nseg, ranks.size), dtype=torch.float32, device="cuda")
        rc = L_.rt_segment_order_stats_device(_lib.ptr(d), B, L * W, L, W, nseg, per_seg, _lib.ptr(ranks),
                                              ranks.size, _lib.ptr(out),
                                              ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        assert rc == 0, L_.rt_last_error()
        got = out.cpu().numpy()
        for b in range(B):
            for iw in range(W):
                for sg in range(nseg):
                    col = snr[b, sg * per_seg:(sg + 1) * per_seg, iw]
                    assert np.array_equal(got[b, iw, sg], np.sort(col)[ranks]), (kind, per_seg, b, iw, sg)


def test_device_find_peaks_long_segments(rt):
    """find_peaks with segments of more than 4096 periods on the device path
    (a wide segwidth), identical to the host computation."""
    import torch
    from riptide_amd import engine
    from riptide_amd.peaks import PeakFinder
    case = inputs.PGRAM_CASES[1]
    plan = engine.PeriodogramPlan.for_search(case["n"], case["tsamp"], case["pmin"], case["pmax"],
                                             case["bmin"], case["bmax"], ducy_max=case["ducy_max"])
    tobs = case["n"] * case["tsamp"]
    periods, _ = plan.grid()
    f = 1.0 / periods
    # a segment width giving segments of ~5000 periods
    segwidth = 5000.0 / plan.length * abs(f[-1] - f[0]) * tobs
    assert 4096 < PeakFinder(plan, tobs, segwidth=segwidth).per_seg <= 32768
    xs = np.stack([inputs.with_signal(case["n"], case["tsamp"], s, 0.41, 14.0) for s in range(2)])
    d = engine.deredden_normalise(torch.from_numpy(xs).cuda(), 1001, 101)
    snr = plan.run(d)
    _device_vs_host_peaks(rt, plan, snr, tobs, segwidth=segwidth, minseg=2)


@pytest.mark.parametrize("name", ["cfg1", "cfg2"])
def test_device_find_peaks_full_config(rt, golden_full, name):
    import torch
    from riptide_amd import engine
    from riptide_amd.peaks import PeakFinder
    g = golden_full["configs"][name]
    c = g["case"]
    raw = inputs.full_input(c)
    if sha(raw) != g["input_sha"]:
        pytest.fail(f"input generator drifted on this host (numpy RNG/libm): input sha256 {sha(raw)} != golden "
                    f"{g['input_sha']}; the full-size parity check cannot run")
    plan = engine.PeriodogramPlan.for_search(c["n"], c["tsamp"], c["pmin"], c["pmax"], c["bmin"], c["bmax"],
                                             ducy_max=c["ducy_max"])
    x = engine.deredden_normalise(torch.from_numpy(raw).cuda(), int(round(4.0 / c["tsamp"])), 101)
    snr = plan.run(x)
    peaks, _ = PeakFinder(plan, c["n"] * c["tsamp"])(snr, dms=[0.0])[0]
    assert [[p.ip, p.iw] for p in peaks] == [[p[0], p[1]] for p in g["peaks"]]   # golden candidate list


# ---------------------------------------------------------------- file input + GPU worker pool
def test_device_sample_conversion_exact(tmp_path):
    import torch
    from riptide_amd.reading import load_device_batch, write_sigproc
    rng = np.random.RandomState(5)
    hdr = {"tsamp": 1e-3, "nbits": 8, "nchans": 1, "refdm": 1.0, "tstart": 58000.0, "src_raj": 0.0,
           "src_dej": 0.0}
    for signed, dtype in ((True, np.int8), (False, np.uint8)):
        data = [rng.randint(np.iinfo(dtype).min, np.iinfo(dtype).max + 1, size=4099).astype(dtype) for _ in range(3)]
        fns = []
        for k, d in enumerate(data):
            fn = str(tmp_path / f"t{int(signed)}_{k}.tim")
            write_sigproc(fn, d, dict(hdr, signed=signed))
            fns.append(fn)
        x, metas, tsamp = load_device_batch(fns, "sigproc")
        assert x.dtype == torch.float32 and tsamp == 1e-3
        for k, d in enumerate(data):
            assert np.array_equal(x[k].cpu().numpy(), d.astype(np.float32))
        assert metas[0]["dm"] == 1.0


# GpuWorkerPool is checked against reference-generated peak lists in
# tests/test_gpu_e2e.py (cfg5 files, the rffa pipeline case).


# ---------------------------------------------------------------- candidate folding
def test_fold_matches_oracle_restatement(rt, oracle):
    from riptide_amd.folding import downsample_rows, fold
    np.random.seed(7)
    ts = rt.TimeSeries.generate(60.0, 1e-3, 0.7317, amplitude=30.0)
    period, bins = 0.7317, 64
    factor = period / bins / ts.tsamp
    # folding.py:65-81 with the oracle's strict downsample
    d = oracle.downsample(ts.data, factor)
    m = d.size // bins
    ref = d[:m * bins].reshape(m, bins).copy()
    ref *= (m * factor) ** -0.5
    assert np.array_equal(fold(ts, period, bins), ref)
    assert np.array_equal(fold(ts, period, bins, subints=1), ref.sum(axis=0))
    sub = fold(ts, period, bins, subints=16)
    cols = np.ascontiguousarray(ref.T)
    exp = np.stack([oracle.downsample(c, m / 16) for c in cols]).T
    assert sub.shape == exp.shape and np.array_equal(sub, exp)
    assert np.argmax(fold(ts, period, bins, subints=1)) in range(bins)
    x = np.random.RandomState(1).normal(size=(5, 1000)).astype(np.float32)
    assert np.array_equal(downsample_rows(x, 3.7), np.stack([oracle.downsample(r, 3.7) for r in x]))
    with pytest.raises(ValueError):
        fold(ts, 1000.0, bins)
    with pytest.raises(ValueError):
        fold(ts, period, 10 ** 6)
    with pytest.raises(ValueError):
        fold(ts, period, bins, subints=10 ** 6)
