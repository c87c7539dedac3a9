"""Generate golden vectors from the REFERENCE implementation (run in the build
container only; /root/reference does not exist on the GPU box).

Sources of truth:
- ``oracle/_ref/native/libcpp*.so``: the reference C++ core (riptide/cpp)
  compiled from its own sources with its own flags by ``make -C oracle ref``;
- the reference's own Python modules for the numpy-level stages
  (running_medians.py, ffautils.py, peak_detection.py, clustering.py,
  timing.py), loaded by file path from /root/reference with ``riptide.libcpp``
  bound to the module above.  Modules that need astropy/schema (absent here)
  are not loaded; the few lines of orchestration they hold (search.py:71-82,
  time_series.py:66-122) are restated below with the same numpy expressions.

Outputs (committed): tests/golden/golden_small.npz (full arrays for reduced
sizes), tests/golden/golden_full.json (digests/statistics/peak lists for the
BASELINE configs at full size).  Inputs are regenerated from
np.random.RandomState(seed) by tests/golden/inputs.py on any machine.

Usage:  python tests/golden/make_golden.py   (needs `make -C oracle ref` first)
"""
import glob
import hashlib
import importlib.util
import json
import os
import platform
import sys
import time
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/riptide"
sys.path.insert(0, HERE)
import inputs  # noqa: E402


def load_reference():
    so = glob.glob(os.path.join(REPO, "oracle", "_ref", "native", "libcpp*.so"))
    if not so:
        raise SystemExit("run `make -C oracle ref` first")
    pkg = types.ModuleType("riptide")
    pkg.__path__ = []
    sys.modules["riptide"] = pkg

    def load(name, path):
        spec = importlib.util.spec_from_file_location("riptide." + name, path)
        mod = importlib.util.module_from_spec(spec)
        sys.modules["riptide." + name] = mod
        setattr(pkg, name, mod)
        spec.loader.exec_module(mod)
        return mod

    load("libcpp", so[0])
    for name in ("timing", "clustering", "ffautils", "running_medians", "peak_detection"):
        load(name, os.path.join(REF, name + ".py"))
    return pkg


class _Pgram:
    """Minimal stand-in for riptide.Periodogram (periodogram.py:9-40) as seen by find_peaks."""

    def __init__(self, widths, periods, foldbins, snrs, tobs, dm):
        self.widths, self.periods, self.foldbins, self.snrs = widths, periods, foldbins, snrs
        self.metadata = {"tobs": tobs, "dm": dm}

    @property
    def freqs(self):
        return 1.0 / self.periods

    @property
    def tobs(self):
        return self.metadata["tobs"]


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def ref_deredden_normalise(R, data, tsamp, rmed_width=4.0, rmed_minpts=101):
    # time_series.py:117-122 then :83-90
    ws = int(round(rmed_width / tsamp))
    rmed = R.running_medians.fast_running_median(data, ws, rmed_minpts)
    x = np.asarray(data - rmed, dtype=np.float32)
    m = x.mean(dtype=np.float64)
    v = x.var(dtype=np.float64)
    return np.asarray((x - m) / v ** 0.5, dtype=np.float32)


def transform_boundary_rows(n, tsamp, pmin, pmax, bmin, bmax):
    """First and last evaluated row of every FFA transform: the plan of
    periodogram.hpp:135-183 (rung ladder, bins loop, rows_eval via ceilshift)
    restated to locate each transform's rows in the periodogram."""
    import math
    f0 = pmin / (tsamp * bmin)
    g = (bmax + 1.0) / bmin
    nds = int(math.ceil(math.log(pmax / pmin) / math.log(g)))
    rows, row = [], 0
    for ids in range(nds):
        f = f0 * g ** ids
        tau = f * tsamp
        nd = int(math.floor(n / f))
        pms = pmax / tau
        bstop = min(bmax, nd, int(pms))
        for b in range(bmin, bstop + 1):
            m = nd // b
            pceil = min(pms, b + 1.0)
            ev = min(m, int(math.ceil(b * (m - 1.0) * (1.0 - b / pceil))))
            if ev > 0:
                rows += [row, row + ev - 1]
            row += ev
    return sorted(set(rows)), row


def main():
    if "--full-only" in sys.argv:
        return main_full(load_reference())
    R = load_reference()
    lc = R.libcpp
    out = {}
    meta = {
        "generated_by": "tests/golden/make_golden.py",
        "reference_build": "g++ -O3 -ffast-math -march=native (setup.py:18)",
        "cpu": platform.processor() or platform.machine(),
        "numpy": np.__version__,
        "python": platform.python_version(),
    }
    try:
        with open("/proc/cpuinfo") as f:
            meta["cpu"] = next(l.split(":", 1)[1].strip() for l in f if l.startswith("model name"))
    except Exception:
        pass

    # (i) ffa2 blocks, bit-exact
    for (m, p, seed) in inputs.FFA_CASES:
        x = inputs.ffa_block(m, p, seed)
        y = lc.ffa2(x)
        key = f"ffa2_{m}x{p}"
        if m * p <= 40_000:
            out[key] = y
        out[key + "_sha"] = np.array(sha(y))
    out["ffa2_88_in"] = inputs.FFA_IN_88
    out["ffa2_88_out"] = lc.ffa2(inputs.FFA_IN_88)

    # (ii) downsample
    x = inputs.noise(20000, 11)
    for f in inputs.DS_FACTORS:
        out[f"downsample_{f!r}"] = lc.downsample(x, f)

    # (iii) snr2 + circular prefix sums
    prof = inputs.noise(200 * 250, 12).reshape(200, 250)
    prof[:, 100:113] += 3.0
    w = np.asarray(inputs.SNR_WIDTHS, dtype=np.uint64)
    out["snr2_out"] = lc.snr2(prof, w, 1.7)
    out["cps_out"] = lc.circular_prefix_sum(prof[0].copy(), 700)

    # (iv) running medians
    x = inputs.noise(1000, 13)
    for wd in inputs.RMED_WIDTHS:
        out[f"rmed_{wd}"] = lc.running_median(x, wd)
    xl = inputs.noise(30011, 14)
    for (ws, mp) in inputs.FAST_RMED_CASES:
        out[f"frmed_{ws}_{mp}"] = R.running_medians.fast_running_median(xl, ws, mp)

    # (v) periodograms at reduced size, data already normalised
    for case in inputs.PGRAM_CASES:
        name = case["name"]
        data = inputs.pgram_input(case)
        widths = R.ffautils.generate_width_trials(case["bmin"], ducy_max=case["ducy_max"], wtsp=1.5)
        t0 = time.time()
        periods, foldbins, snrs = lc.periodogram(data, case["tsamp"], widths, case["pmin"],
                                                 case["pmax"], case["bmin"], case["bmax"])
        out[f"pg_{name}_widths"] = np.asarray(widths)
        out[f"pg_{name}_periods"] = periods
        out[f"pg_{name}_foldbins"] = foldbins
        out[f"pg_{name}_snrs"] = snrs
        out[f"pg_{name}_input_sha"] = np.array(sha(data))
        print(f"pgram {name}: L={periods.size} ({time.time()-t0:.2f}s)")

    # (v-b) full ffa_search pipeline (deredden + normalise + periodogram) at reduced size
    for case in inputs.SEARCH_CASES:
        name = case["name"]
        raw = inputs.search_input(case)
        x = ref_deredden_normalise(R, raw, case["tsamp"], case["rmed_width"], case["rmed_minpts"])
        widths = R.ffautils.generate_width_trials(case["bmin"], ducy_max=case["ducy_max"], wtsp=1.5)
        periods, foldbins, snrs = lc.periodogram(x, case["tsamp"], widths, case["pmin"],
                                                 case["pmax"], case["bmin"], case["bmax"])
        out[f"search_{name}_normalised_sha"] = np.array(sha(x))
        out[f"search_{name}_normalised_head"] = x[:4096]
        out[f"search_{name}_snrs"] = snrs
        out[f"search_{name}_periods_sha"] = np.array(sha(periods))
        out[f"search_{name}_input_sha"] = np.array(sha(raw))
        pg = _Pgram(widths, periods, foldbins, snrs, raw.size * case["tsamp"], 0.0)
        peaks, _ = R.peak_detection.find_peaks(pg)
        out[f"search_{name}_peaks"] = np.array([(p.ip, p.iw, p.snr) for p in peaks], dtype=np.float64).reshape(-1, 3)

    np.savez_compressed(os.path.join(HERE, "golden_small.npz"), **out)
    main_full(R, meta)


def main_full(R, meta=None):
    """(vi) full-size BASELINE configs: digests, per-width statistics, 5000
    sampled rows plus the first and last evaluated row of every transform,
    and the find_peaks list."""
    if meta is None:
        with open(os.path.join(HERE, "golden_full.json")) as f:
            meta = json.load(f)["meta"]
    lc = R.libcpp
    full = {"meta": meta, "configs": {}}
    for case in inputs.FULL_CASES:
        name = case["name"]
        t0 = time.time()
        raw = inputs.full_input(case)
        x = ref_deredden_normalise(R, raw, case["tsamp"])
        widths = R.ffautils.generate_width_trials(case["bmin"], ducy_max=case["ducy_max"], wtsp=1.5)
        t1 = time.time()
        periods, foldbins, snrs = lc.periodogram(x, case["tsamp"], widths, case["pmin"],
                                                 case["pmax"], case["bmin"], case["bmax"])
        t2 = time.time()
        pg = _Pgram(widths, periods, foldbins, snrs, raw.size * case["tsamp"], 0.0)
        peaks, _ = R.peak_detection.find_peaks(pg)
        t3 = time.time()
        bounds, total = transform_boundary_rows(case["n"], case["tsamp"], case["pmin"], case["pmax"],
                                                case["bmin"], case["bmax"])
        assert total == periods.size
        rows = np.union1d(inputs.sample_rows(periods.size, count=5000), np.asarray(bounds, dtype=np.int64))
        full["configs"][name] = {
            "case": case,
            "input_sha": sha(raw),
            "normalised_sha": sha(x),
            "widths": [int(w) for w in widths],
            "length": int(periods.size),
            "periods_sha": sha(periods),
            "foldbins_sha": sha(foldbins),
            "snr_max": [float(v) for v in snrs.max(axis=0)],
            "snr_argmax": [int(v) for v in snrs.argmax(axis=0)],
            "snr_sum": [float(v) for v in snrs.astype(np.float64).sum(axis=0)],
            "snr_abs_sum": [float(v) for v in np.abs(snrs.astype(np.float64)).sum(axis=0)],
            "boundary_rows": [int(r) for r in bounds],
            "sample_rows": [int(r) for r in rows],
            "sample_snrs": snrs[rows].astype(float).tolist(),
            "peaks": [[int(p.ip), int(p.iw), float(p.snr)] for p in peaks],
            "seconds": {"deredden_normalise": t1 - t0, "periodogram": t2 - t1, "find_peaks": t3 - t2},
        }
        print(f"full {name}: L={periods.size} peaks={len(peaks)} pgram={t2-t1:.2f}s peaks={t3-t2:.2f}s")
    with open(os.path.join(HERE, "golden_full.json"), "w") as f:
        json.dump(full, f, separators=(",", ":"))


if __name__ == "__main__":
    main()
