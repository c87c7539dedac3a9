"""CPU baseline for bench.py (TEST INFRASTRUCTURE, run in a subprocess).

The rffa CPU model (riptide/pipeline/worker_pool.py:35-45 and
pipeline.py:508): a multiprocessing.Pool of C worker processes, one DM trial
per process, BLAS pinned to one thread; each trial is dereddened and
normalised (numpy, restated in oracle.py from time_series.py:66-122), then
searched by the reference C++ periodogram built from the reference sources
with its own flags (oracle/_ref/v4 = -march=x86-64-v4 on AVX-512 hosts,
oracle/_ref/portable = x86-64-v3 otherwise -> kind "reference"; the clean-room
C restatement when neither is present -> kind "port"), then run through
find_peaks (riptide_amd.peak_detection, the reference's numpy expressions).

C = the worker processes actually used: the CPU share this process may use
(sched_getaffinity, capped by OMP_NUM_THREADS where the harness sets it, as on
the GPU box: 16 host cores per GPU).  Reports the search-only rate (deredden
+ normalise + periodogram: the work bench.py's GPU step does) as `value`, and
search + find_peaks separately.  Prints one JSON object.
"""
import argparse
import glob
import importlib.util
import json
import multiprocessing
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# run as a script: drop oracle/ itself from the path so `oracle` is the package
sys.path = [p for p in sys.path if os.path.abspath(p or '.') != HERE]
sys.path.insert(0, os.path.dirname(HERE))

_A = None            # parsed arguments (inherited by the forked workers)
_PGRAM = None
_KIND = None


def _avx512():
    try:
        with open("/proc/cpuinfo") as f:
            return any(l.startswith("flags") and " avx512f" in l for l in f)
    except OSError:
        return False


def _load_pgram():
    from oracle import oracle as O
    for sub in (["v4"] if _avx512() else []) + ["portable"]:
        so = glob.glob(os.path.join(HERE, "_ref", sub, "libcpp*.so"))
        if so:
            try:
                spec = importlib.util.spec_from_file_location("libcpp", so[0])
                mod = importlib.util.module_from_spec(spec)
                spec.loader.exec_module(mod)
                return mod.periodogram, "reference", f"reference C++ (-O3 -ffast-math, {sub} build)"
            except Exception:
                pass
    O.build()
    return (lambda d, ts, w, p0, p1, b0, b1: O.periodogram(d, ts, w, p0, p1, b0, b1)), "port", "oracle C restatement"


def _trial(k):
    """One DM trial (process_fname model): returns absolute timestamps
    (start, search done, peaks done) after the untimed input generation."""
    from oracle import oracle as O
    from riptide_amd.peak_detection import find_peaks
    from riptide_amd.periodogram import Periodogram
    a = _A
    raw = np.random.RandomState(1234 + k).normal(size=a.n).astype(np.float32)
    widths = O.generate_width_trials(a.bmin, a.ducy_max)
    t0 = time.time()
    x = O.normalise(O.deredden(raw, a.tsamp, 4.0, 101))
    periods, foldbins, snrs = _PGRAM(x, a.tsamp, widths, a.pmin, a.pmax, a.bmin, a.bmax)
    t1 = time.time()
    pg = Periodogram(widths, periods, foldbins, snrs, metadata={"tobs": a.n * a.tsamp, "dm": float(k)})
    find_peaks(pg)
    t2 = time.time()
    return t0, t1, t2


def default_cores():
    c = len(os.sched_getaffinity(0))
    for var in ("OMP_NUM_THREADS",):
        v = os.environ.get(var)
        if v and v.isdigit() and int(v) > 0:
            c = min(c, int(v))
    return c


def main():
    global _A, _PGRAM, _KIND
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 23)
    ap.add_argument("--tsamp", type=float, default=256e-6)
    ap.add_argument("--pmin", type=float, default=0.1)
    ap.add_argument("--pmax", type=float, default=10.0)
    ap.add_argument("--bmin", type=int, default=240)
    ap.add_argument("--bmax", type=int, default=260)
    ap.add_argument("--ducy-max", type=float, default=0.05)
    ap.add_argument("--cores", type=int, default=0, help="worker processes (default: this process's CPU share)")
    ap.add_argument("--trials-per-core", type=int, default=1)
    _A = ap.parse_args()
    cores = _A.cores or default_cores()
    for var in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS"):   # threadpool_limits(1)
        os.environ[var] = "1"
    ntrials = cores * _A.trials_per_core
    _PGRAM, _KIND, what = _load_pgram()
    ctx = multiprocessing.get_context("fork")
    with ctx.Pool(processes=cores) as pool:
        stamps = pool.map(_trial, range(ntrials), chunksize=1)
    start = min(s[0] for s in stamps)
    search_wall = max(s[1] for s in stamps) - start
    total_wall = max(s[2] for s in stamps) - start
    print(json.dumps({
        "value": ntrials / search_wall, "unit": "DM trials/s", "cores": cores, "kind": _KIND,
        "search_and_peaks_per_s": ntrials / total_wall,
        "per_core_search_per_s": ntrials / search_wall / cores,
        "sample": f"{ntrials} cfg2 trial(s) of {_A.n} samples, multiprocessing.Pool({cores}) one trial per "
                  f"process (rffa worker-pool model): numpy deredden+normalise + {what} periodogram = value; "
                  f"+ find_peaks = search_and_peaks_per_s; host CPU share {len(os.sched_getaffinity(0))} "
                  f"affinity cores",
        "seconds": total_wall}))


if __name__ == "__main__":
    main()
