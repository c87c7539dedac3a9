"""CPU-only tests: the C-ABI library loads and exports every symbol of
include/riptide_amd.h; the host planner (ladder, trial grid, pass schedule) is
bit-exact with the reference; host-side Python logic (width trials, ffafreq,
clustering, peak detection, argument validation) matches the reference.
No compute call reaches the GPU here."""
import ctypes
import hashlib
import os
import re

import numpy as np
import pytest

import inputs
from conftest import REPO

HEADER = os.path.join(REPO, "include", "riptide_amd.h")


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.fixture(scope="module")
def lib():
    from riptide_amd import _lib
    return _lib.load()


def test_header_symbols_exported(lib):
    text = open(HEADER).read()
    declared = set(re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\**(rt_\w+)\s*\(", text, re.M))
    assert len(declared) >= 25
    from riptide_amd import _lib
    for name in declared:
        assert hasattr(lib, name), name
        assert name in _lib.EXPORTED, f"{name} has no ctypes signature"
    # and nothing in the loader that the header does not declare
    assert set(_lib.EXPORTED) <= declared


def test_test_hooks_only_in_test_build(lib):
    """The fault-injection entry point is not part of the product library;
    the test build (libriptide_amd_testhooks.so) carries it."""
    import ctypes as ct
    from riptide_amd import _lib
    assert not hasattr(lib, "rt_test_corrupt_next_plans")
    assert "rt_test_corrupt_next_plans" not in _lib.EXPORTED
    t = ct.CDLL(_lib.TESTHOOKS_PATH, mode=ct.RTLD_LOCAL)
    assert hasattr(t, "rt_test_corrupt_next_plans")
    text = open(os.path.join(os.path.dirname(HEADER), "riptide_amd_test.h")).read()
    assert "int rt_test_corrupt_next_plans(int on);" in text


def _ladder(lib, n, c):
    fused = ctypes.c_int(-1)
    rungs = ctypes.c_uint64()
    rc = lib.rt_ladder_check(n, c["tsamp"], c["pmin"], c["pmax"], c["bmin"], c["bmax"], ctypes.byref(fused),
                             ctypes.byref(rungs))
    assert rc == 0, lib.rt_last_error()
    return fused.value, rungs.value


def test_ladder_path_choice(lib):
    """The fused ladder indexes samples in 32 bits: series of 2^29 samples or
    more take the per-rung (64-bit) kernel (the planner enforces
    the fused kernel's index range instead of assuming it)."""
    c = dict(tsamp=256e-6, pmin=0.1, pmax=10.0, bmin=240, bmax=260)
    assert _ladder(lib, 1 << 23, c)[0] == 1            # cfg2: fused
    assert _ladder(lib, (1 << 29) - 1, c)[0] == 1
    assert _ladder(lib, 1 << 29, c)[0] == 0            # 2^29: per-rung
    assert _ladder(lib, (1 << 30) + 7, c)[0] == 0
    f, r = _ladder(lib, 1 << 23, c)
    assert r > 0
    # with the 512-float margin every BASELINE config and cfg5's
    # short / medium ranges still take the fused ladder (cfg4's largest factor
    # is ~310); cfg5's long range (factors up to ~1950) takes the fused ladder
    # for its rungs inside the margin and the per-rung kernel for the rest (2)
    cfg4 = dict(tsamp=64e-6, pmin=0.002, pmax=0.5, bmin=16, bmax=32)
    assert _ladder(lib, 1 << 22, cfg4)[0] == 1
    assert _ladder(lib, 2343750, dict(tsamp=256e-6, pmin=0.5, pmax=2.0, bmin=240, bmax=260))[0] == 1   # cfg1
    assert _ladder(lib, 1 << 22, dict(tsamp=256e-6, pmin=0.2, pmax=5.0, bmin=240, bmax=260))[0] == 1   # cfg3
    for rng in inputs.CFG5["ranges"]:
        s = rng["ffa_search"]
        want = 2 if rng["name"] == "long" else 1
        assert _ladder(lib, inputs.CFG5["n"], dict(tsamp=inputs.CFG5["tsamp"], pmin=s["period_min"],
                                                   pmax=s["period_max"], bmin=s["bins_min"],
                                                   bmax=s["bins_max"]))[0] == want, rng["name"]
    # the margin's edge: largest factor with ceil(f) + 2 == 512 is fused,
    # one more sample of window is not (that rung alone to the per-rung kernel)
    assert _ladder(lib, 1 << 20, inputs.LADDER_EDGE_CASE)[0] == 1
    over = dict(inputs.LADDER_EDGE_CASE, pmin=inputs.LADDER_EDGE_CASE["pmin"] * 510.5 / 509.5125)
    over["pmax"] = over["pmin"] * 1.125 ** 2 * 0.999
    assert _ladder(lib, 1 << 20, over)[0] in (0, 2)
    # every rung past the margin: nothing for the fused kernel
    assert _ladder(lib, 1 << 22, dict(tsamp=64e-6, pmin=40.0, pmax=100.0, bmin=960, bmax=1040))[0] == 0


def test_version(lib):
    assert b"gfx950" in lib.rt_version()


def _grid(lib, c):
    L = ctypes.c_size_t()
    rc = lib.rt_periodogram_length(c["n"], c["tsamp"], c["pmin"], c["pmax"], c["bmin"], c["bmax"], ctypes.byref(L))
    assert rc == 0
    periods = np.empty(L.value, np.float64)
    foldbins = np.empty(L.value, np.uint32)
    from riptide_amd._lib import ptr
    assert lib.rt_periodogram_grid(c["n"], c["tsamp"], c["pmin"], c["pmax"], c["bmin"], c["bmax"],
                                   ptr(periods), ptr(foldbins)) == 0
    return periods, foldbins


@pytest.mark.parametrize("case", inputs.PGRAM_CASES, ids=lambda c: c["name"])
def test_grid_small_bit_exact(lib, golden, case):
    periods, foldbins = _grid(lib, case)
    assert np.array_equal(periods, golden[f"pg_{case['name']}_periods"])
    assert np.array_equal(foldbins, golden[f"pg_{case['name']}_foldbins"])


@pytest.mark.parametrize("name", ["cfg1", "cfg2", "cfg3", "cfg4"])
def test_grid_full_bit_exact(lib, golden_full, name):
    g = golden_full["configs"][name]
    periods, foldbins = _grid(lib, g["case"])
    assert periods.size == g["length"]
    assert sha(periods) == g["periods_sha"]
    assert sha(foldbins) == g["foldbins_sha"]


@pytest.mark.parametrize("case", inputs.FULL_CASES + inputs.PGRAM_CASES + inputs.SEARCH_CASES,
                         ids=lambda c: c["name"] + str(c["n"]))
def test_schedule_invariants(lib, case):
    u = [ctypes.c_uint64() for _ in range(4)]
    d = [ctypes.c_double() for _ in range(2)]
    rc = lib.rt_schedule_check(case["n"], case["tsamp"], 10, case["pmin"], case["pmax"], case["bmin"], case["bmax"],
                               ctypes.byref(u[0]), ctypes.byref(u[1]), ctypes.byref(u[2]), ctypes.byref(d[0]),
                               ctypes.byref(d[1]), ctypes.byref(u[3]))
    assert rc == 0, lib.rt_last_error()
    assert u[1].value >= u[0].value > 0
    # actual traffic stays within 1.6x the SURVEY.md §8(d) algorithmic bytes
    assert d[1].value <= 1.6 * d[0].value


def test_schedule_cfg2_shape(lib):
    """cfg2 (headline): every cell of every transform is transformed; the plan
    has the documented size (1153 transforms, 1331.6 M cells)."""
    u = [ctypes.c_uint64() for _ in range(4)]
    d = [ctypes.c_double() for _ in range(2)]
    assert lib.rt_schedule_check(1 << 23, 256e-6, 6, 0.1, 10.0, 240, 260, *(ctypes.byref(x) for x in u[:3]),
                                 ctypes.byref(d[0]), ctypes.byref(d[1]), ctypes.byref(u[3])) == 0
    assert u[0].value == 1153
    assert abs(u[3].value / 1e6 - 1331.6) < 0.1


def test_schedule_refuses_blocks_over_2gib(lib):
    """A transform block of >= 2^31 bytes would overflow the cone kernel's
    32-bit buffer range: the planner refuses it with ValueError
    text instead of producing silently wrong output.  f == 1 rung: m * p = N."""
    u = [ctypes.c_uint64() for _ in range(4)]
    d = [ctypes.c_double() for _ in range(2)]
    args = (*(ctypes.byref(x) for x in u[:3]), ctypes.byref(d[0]), ctypes.byref(d[1]), ctypes.byref(u[3]))
    n = (1 << 29) + 4096                       # 2^31 + 16 KiB of samples at the first rung
    rc = lib.rt_schedule_check(n, 1e-3, 2, 0.24, 0.3, 240, 260, *args)
    assert rc == 1 and b"2 GiB" in lib.rt_last_error()
    n = (1 << 29) - 4096 * 260                 # every block below 2 GiB
    assert lib.rt_schedule_check(n, 1e-3, 2, 0.24, 0.25, 240, 240, *args) == 0, lib.rt_last_error()


def test_periodogram_length_errors(lib):
    from riptide_amd import _lib
    L = ctypes.c_size_t()
    cases = [(0.0, 1.0, 2.0, 240, 260, "tsamp must be > 0"),
             (1e-3, 0.0, 2.0, 240, 260, "period_min must be > 0"),
             (1e-3, 1.0, 0.5, 240, 260, "period_max must be > period_min"),
             (1e-3, 1.0, 2.0, 1, 260, "bins_min must be > 1"),
             (1e-3, 1.0, 2.0, 240, 200, "bins_max must be >= bins_min"),
             (1e-3, 0.1, 2.0, 240, 260, "Must have: period_min >= tsamp * bins_min")]
    for tsamp, pmin, pmax, bmin, bmax, msg in cases:
        rc = lib.rt_periodogram_length(10000, tsamp, pmin, pmax, bmin, bmax, ctypes.byref(L))
        assert rc == _lib.RT_EINVAL
        assert lib.rt_last_error().decode().startswith(msg)


def test_width_trials():
    from riptide_amd import generate_width_trials
    assert list(generate_width_trials(240, ducy_max=0.05)) == [1, 2, 3, 4, 6, 9]
    assert list(generate_width_trials(240)) == [1, 2, 3, 4, 6, 9, 13, 19, 28, 42]
    assert list(generate_width_trials(16)) == [1, 2, 3]


def test_ffafreq():
    # test_ffa_base_functions.py:78-118
    from riptide_amd import ffafreq, ffaprd
    m, p = 42, 127
    dt = np.pi / 1000.0
    s = np.arange(m, dtype=float)
    true_periods = p ** 2 / (p - s / (m - 1.0)) * dt
    assert np.allclose(ffafreq(m * p, p, dt=dt), 1.0 / true_periods)
    assert np.allclose(ffaprd(m * p, p, dt=dt), true_periods)
    assert ffafreq(p, p, dt=dt)[0] == 1.0 / (p * dt)
    for args in ((0, p), (np.pi, p), (m * p, 1), (m * p, np.pi), (m * p, m * p + 1)):
        with pytest.raises(ValueError):
            ffafreq(*args, dt=dt)
    with pytest.raises(ValueError):
        ffafreq(m * p, p, dt=0)


def test_cluster1d():
    from riptide_amd import cluster1d
    assert cluster1d(np.array([]), 1.0) == []
    x = np.array([5.0, 1.0, 1.5, 9.0, 5.2])
    cl = cluster1d(x, 0.6)
    assert [sorted(c.tolist()) for c in cl] == [[1, 2], [0, 4], [3]]
    assert [c.tolist() for c in cluster1d(np.array([1.0, 1.1, 1.2]), 0.5)] == [[0, 1, 2]]


def test_find_peaks_on_reference_snr(golden):
    """Host peak detection on the REFERENCE's S/N reproduces the reference's
    candidate list exactly (the logic is unchanged; see peak_detection.py)."""
    from riptide_amd import Metadata, Periodogram, find_peaks
    for case in inputs.SEARCH_CASES:
        name = case["name"]
        from riptide_amd._lib import load, ptr
        lib = load()
        L = ctypes.c_size_t()
        lib.rt_periodogram_length(case["n"], case["tsamp"], case["pmin"], case["pmax"], case["bmin"],
                                  case["bmax"], ctypes.byref(L))
        periods = np.empty(L.value)
        foldbins = np.empty(L.value, np.uint32)
        lib.rt_periodogram_grid(case["n"], case["tsamp"], case["pmin"], case["pmax"], case["bmin"], case["bmax"],
                                ptr(periods), ptr(foldbins))
        snrs = golden[f"search_{name}_snrs"]
        from riptide_amd import generate_width_trials
        widths = generate_width_trials(case["bmin"], ducy_max=case["ducy_max"])
        pg = Periodogram(widths, periods, foldbins, snrs, metadata=Metadata({"tobs": case["n"] * case["tsamp"],
                                                                             "dm": 0.0}))
        peaks, _ = find_peaks(pg)
        got = np.array([(p.ip, p.iw, p.snr) for p in peaks], dtype=np.float64).reshape(-1, 3)
        assert np.array_equal(got, golden[f"search_{name}_peaks"])


def test_shim_validation_before_device():
    """Argument errors of the drop-in are raised before any device work."""
    from riptide_amd import libcpp
    with pytest.raises(ValueError, match="contiguous"):
        libcpp.ffa2(np.zeros((8, 8), np.float32)[:, ::2])
    with pytest.raises(ValueError, match="incorrect number of dimensions"):
        libcpp.ffa2(np.zeros(8, np.float32))
    with pytest.raises(ValueError, match="same number of elements"):
        libcpp.fused_rollback_add(np.zeros(3), np.zeros(4), 1)
    with pytest.raises(ValueError, match="Downsampling factor"):
        libcpp.downsample(np.zeros(10, np.float32), 0.5)


def test_periodogram_object():
    from riptide_amd import Metadata, Periodogram
    pg = Periodogram(np.array([1, 2]), np.array([1.0, 2.0]), np.array([240, 240], np.uint32),
                     np.zeros((2, 2), np.float32), metadata=Metadata({"tobs": 10.0}))
    assert np.array_equal(pg.freqs, [1.0, 0.5])
    assert pg.tobs == 10.0
    assert Periodogram.from_dict(pg.to_dict()).metadata == pg.metadata
    assert Metadata({})["dm"] is None


def test_ffa_schedules_validate(lib):
    """The pass schedule rt_ffa2 runs for every golden FFA shape, plus edge
    shapes (one row, short / long rows, node sizes around the LDS capacity),
    passes the host validation the kernel relies on (unit blobs: DMA
    segments tile the fill, row-slot tables cover every row once, row pairs
    share head and tail rows)."""
    from tests.golden import inputs
    shapes = {(m, p) for m, p, _ in inputs.FFA_CASES}
    shapes |= {(1, 1), (1, 260), (2, 1), (3, 17), (64, 32), (65, 33), (384, 16), (385, 16), (1000, 31),
               (72, 250), (73, 250), (5000, 257), (4097, 64), (300, 700), (40, 2880)}
    n = ctypes.c_uint64()
    for m, p in sorted(shapes):
        assert lib.rt_ffa_schedule_check(m, p, ctypes.byref(n)) == 0, (m, p, lib.rt_last_error())
        assert n.value >= 1
    assert lib.rt_ffa_schedule_check(0, 16, None) == 1


# ---------------------------------------------------------------- host sanitizers
def _asan_cases():
    from riptide_amd.ffautils import generate_width_trials
    cases = []
    for c in inputs.FULL_CASES:
        w = len(generate_width_trials(c["bmin"], ducy_max=c["ducy_max"], wtsp=1.5))
        cases.append((c["name"], ["pgram", c["n"], c["tsamp"], c["pmin"], c["pmax"], c["bmin"], c["bmax"], w], {}))
    c2 = inputs.FULL_CASES[1]
    w2 = len(generate_width_trials(c2["bmin"], ducy_max=c2["ducy_max"], wtsp=1.5))
    cases.append(("cfg2-bench-1536M", ["pgram", c2["n"], c2["tsamp"], c2["pmin"], c2["pmax"], c2["bmin"], c2["bmax"], w2],
                  {"RIPTIDE_AMD_SCRATCH_MFLOATS": "1536"}))
    cases.append(("cfg2-cosched-384M", ["pgram", c2["n"], c2["tsamp"], c2["pmin"], c2["pmax"], c2["bmin"], c2["bmax"], w2],
                  {"RIPTIDE_AMD_SCRATCH_MFLOATS": "384", "RIPTIDE_AMD_COSCHED": "1"}))
    c5 = inputs.CFG5
    for r in c5["ranges"]:
        f = r["ffa_search"]
        w = len(generate_width_trials(f["bins_min"], ducy_max=0.2, wtsp=f["wtsp"]))
        cases.append((f"cfg5-{r['name']}", ["pgram", c5["n"], c5["tsamp"], f["period_min"], f["period_max"],
                                            f["bins_min"], f["bins_max"], w], {}))
    for m, p in [(1, 1), (2, 1), (7, 3), (33, 64), (150, 260), (1023, 34), (1025, 34), (5000, 260), (21474, 240),
                 (134217, 16), (3000, 17), (777, 4000), (40, 12000), (9, 70000),
                 (999, 9), (1500, 12), (5000, 20), (4099, 24), (2049, 27), (3001, 31), (65537, 32)]:
        cases.append((f"ffa-{m}x{p}", ["ffa", m, p], {}))
    for m, p, _ in inputs.FFA_CASES:
        cases.append((f"ffa-{m}x{p}", ["ffa", m, p], {}))
    return cases


def test_asan_schedule_check():
    """The host planner and the C ABI's host-only entry points under
    AddressSanitizer + UBSan (`make -C riptide_amd/csrc asan`): the period
    grid, the pass schedule with every unit blob / DMA segment table /
    row-slot table (validate_exec_plan), and the ladder choice, for the five
    BASELINE configurations (cfg2 also at bench.py's one-group budget), and
    the single-transform schedules of every ffa2 shape the GPU parity tests
    run.  Any sanitizer report aborts the checker (exit status != 0)."""
    import subprocess
    from concurrent.futures import ThreadPoolExecutor
    exe = os.path.join(REPO, "build", "asan", "sched_check")
    subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "riptide_amd", "csrc"), "asan"])
    env0 = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=99",
                UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    # ffa shapes whose rows are too wide for the LDS engine (p > 45 x 64
    # bins) take the global-memory path: rt_ffa_schedule_check rejects them

    def run(case):
        name, argv, extra = case
        env = {k: v for k, v in env0.items() if k not in ("RIPTIDE_AMD_SCRATCH_MFLOATS", "RIPTIDE_AMD_COSCHED")}
        env.update(extra)
        r = subprocess.run([exe] + [str(a) for a in argv], env=env, capture_output=True, text=True, timeout=600)
        return name, argv, r

    cases = _asan_cases()
    with ThreadPoolExecutor(max_workers=min(6, os.cpu_count() or 2)) as ex:
        results = list(ex.map(run, cases))
    for name, argv, r in results:
        assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, (name, r.stderr[-3000:])
        if argv[0] == "ffa" and argv[2] > 45 * 64:
            assert r.returncode == 1 and "bad shape" in r.stdout, (name, r.stdout, r.stderr[-2000:])
            continue
        assert r.returncode == 0, (name, r.returncode, r.stdout, r.stderr[-3000:])
        if name == "cfg2-bench-1536M":
            assert int(r.stdout.split("launches=")[1].split()[0]) <= 16, r.stdout


def test_bench_pmc_summary_matches_sources(tmp_path, monkeypatch):
    """bench.pmc_traffic takes the newest PMC summary measured on the current
    kernel sources (csrc_sha == source_digest()), not merely the newest file
    name, and reports the traffic as stale when none matches."""
    import json
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    (tmp_path / "riptide_amd" / "csrc").mkdir(parents=True)
    (tmp_path / "riptide_amd" / "csrc" / "k.hip").write_text("kernel v1")
    (tmp_path / "profiles").mkdir()
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    cur = bench.source_digest()

    def put(name, sha, hbm):
        (tmp_path / "profiles" / name).write_text(json.dumps({"csrc_sha": sha, "hbm_bytes_per_trial": hbm}))

    put("r06a_pmc_cone.json", "0123", 1.0)
    put("r06f_pmc_cone.json", cur, 2.0)
    put("r06z_pmc_cone.json", "4567", 3.0)           # newest name, other sources
    s, why = bench.pmc_traffic("cfg2")
    assert why == "ok" and s["hbm_bytes_per_trial"] == 2.0 and s["source"].endswith("r06f_pmc_cone.json")
    put("r06f_pmc_cone_cfg3.json", "0123", 1.0)
    s, why = bench.pmc_traffic("cfg3")
    assert s is None and why.startswith("stale")
