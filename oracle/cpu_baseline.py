"""CPU baseline for bench.py (TEST INFRASTRUCTURE, run in a subprocess).

The rffa CPU model (riptide/pipeline/worker_pool.py:35-70 and
pipeline.py:508): a multiprocessing.Pool of C worker processes, one DM trial
per process, BLAS pinned to one thread; each trial is dereddened and
normalised (numpy, restated in oracle.py from time_series.py:66-122), then
searched by the reference C++ periodogram built from the reference sources
with its own flags (oracle/_ref/v4 = -march=x86-64-v4 on AVX-512 hosts,
oracle/_ref/portable = x86-64-v3 otherwise -> kind "reference"; the clean-room
C restatement when neither is present -> kind "port"), then run through
find_peaks (riptide_amd.peak_detection, the reference's numpy expressions).

Workloads (bench.py legs):
  cfg2  one 2^23-sample trial per process (P 0.1-10 s, bins 240-260, W 6);
  cfg3  one 2^22-sample trial per process (P 0.2-5 s, bins 240-260, W 10);
  cfg5  SIGPROC files (--files-from, one path a line) searched like
        WorkerPool.process_fname: read, deredden + normalise once, then every
        example.yaml range (periodogram + find_peaks).

C = the worker processes used: `--cores N`, `--cores all` (every core of
sched_getaffinity that a cgroup CPU quota lets this process use -- the
node-level comparison on a dedicated host), or by default this process's CPU
share (sched_getaffinity capped by OMP_NUM_THREADS where the harness sets it,
and by the CPU quota: 16 host cores per GPU on the GPU box).  Workers are also capped so their
resident memory (measured ~0.5 GB per cfg2 trial) stays within half of the
available memory and 120 GB.  Reports the search-only rate (deredden + normalise +
periodogram: the work bench.py's GPU step does) as `value`, and search +
find_peaks separately.  Prints one JSON object.
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
_FILES = []

WORKLOADS = {
    "cfg2": dict(n=1 << 23, tsamp=256e-6, pmin=0.1, pmax=10.0, bmin=240, bmax=260, ducy_max=0.05),
    "cfg3": dict(n=1 << 22, tsamp=256e-6, pmin=0.2, pmax=5.0, bmin=240, bmax=260, ducy_max=0.2),
}
# cfg5: tests/golden/inputs.py CFG5 (example.yaml's dereddening and ranges)
CFG5_DEREDDEN = (5.0, 101)
CFG5_RANGES = [(0.2, 0.5, 240, 260), (0.5, 2.0, 480, 520), (2.0, 120.0, 960, 1040)]
RSS_GB = {"cfg2": 0.55, "cfg3": 0.35, "cfg5": 0.9}


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
    """One synthetic DM trial (process_fname model): returns absolute
    timestamps (start, search done, peaks done) after the untimed input
    generation."""
    from oracle import oracle as O
    from riptide_amd.peak_detection import find_peaks
    from riptide_amd.periodogram import Periodogram
    c = WORKLOADS[_A.workload]
    raw = np.random.RandomState(1234 + k).normal(size=c["n"]).astype(np.float32)
    widths = O.generate_width_trials(c["bmin"], c["ducy_max"])
    t0 = time.time()
    x = O.normalise(O.deredden(raw, c["tsamp"], 4.0, 101))
    periods, foldbins, snrs = _PGRAM(x, c["tsamp"], widths, c["pmin"], c["pmax"], c["bmin"], c["bmax"])
    t1 = time.time()
    pg = Periodogram(widths, periods, foldbins, snrs, metadata={"tobs": c["n"] * c["tsamp"], "dm": float(k)})
    find_peaks(pg)
    t2 = time.time()
    return t0, t1, t2


def _file(k):
    """WorkerPool.process_fname (worker_pool.py:47-70) on file k: the read is
    inside the timed region, as in rffa; the search time (read + deredden +
    normalise + periodograms) and the find_peaks time are kept apart."""
    from oracle import oracle as O
    from riptide_amd.peak_detection import find_peaks
    from riptide_amd.periodogram import Periodogram
    from riptide_amd.reading import read_sigproc
    t0 = time.time()
    data, meta, tsamp = read_sigproc(_FILES[k])
    x = O.normalise(O.deredden(np.asarray(data, np.float32), tsamp, *CFG5_DEREDDEN))
    tobs = x.size * tsamp
    search = peaks = 0.0
    for pmin, pmax, bmin, bmax in CFG5_RANGES:
        a = time.time()
        widths = O.generate_width_trials(bmin, 0.2, 1.5)
        periods, foldbins, snrs = _PGRAM(x, tsamp, widths, pmin, pmax, bmin, bmax)
        b = time.time()
        find_peaks(Periodogram(widths, periods, foldbins, snrs, metadata={"tobs": tobs, "dm": meta.get("dm")}),
                   smin=6.0)
        search += b - a
        peaks += time.time() - b
    t1 = time.time()
    # (start, search done, peaks done) on the trial's own clock: find_peaks
    # time moved to the end so the search stamp counts read + search only
    return t0, t1 - peaks, t1


def cpu_quota():
    """Cores' worth of CPU time this process's cgroup may use (cgroup v2
    cpu.max or v1 cfs quota), or None when unlimited / unknown.  A shared
    GPU box shows every core in the affinity mask but grants a share."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            return float(q) / float(per)
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        if q > 0:
            return q / per
    except (OSError, ValueError):
        pass
    return None


def default_cores():
    c = len(os.sched_getaffinity(0))
    for var in ("OMP_NUM_THREADS",):
        v = os.environ.get(var)
        if v and v.isdigit() and int(v) > 0:
            c = min(c, int(v))
    q = cpu_quota()
    if q:
        c = min(c, max(1, int(q)))
    return c


def _mem_available_gb():
    try:
        with open("/proc/meminfo") as f:
            for line in f:
                if line.startswith("MemAvailable:"):
                    return int(line.split()[1]) / 2 ** 20
    except OSError:
        pass
    return None


def main():
    global _A, _PGRAM, _KIND, _FILES
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", choices=("cfg2", "cfg3", "cfg5"), default="cfg2")
    ap.add_argument("--cores", default="", help="worker processes: N, 'all' (every affinity core), "
                                                "default this process's CPU share")
    ap.add_argument("--trials-per-core", type=int, default=1)
    ap.add_argument("--files-from", default="", help="cfg5: text file with one SIGPROC path per line")
    _A = ap.parse_args()
    affinity = len(os.sched_getaffinity(0))
    quota = cpu_quota()
    if _A.cores == "all":
        # every core this process may really use: the affinity mask, capped
        # by a cgroup CPU quota (running more workers than the quota only
        # time-slices them)
        cores = min(affinity, max(1, int(quota))) if quota else affinity
    elif _A.cores:
        cores = int(_A.cores)
    else:
        cores = default_cores()
    mem = _mem_available_gb()
    mem_cap = None
    if mem:
        # half the available memory, at most 120 GB (the GPU box's per-command cap is 270 GB)
        mem_cap = max(1, int(min(0.5 * mem, 120.0) / RSS_GB[_A.workload]))
        cores = min(cores, mem_cap)
    for var in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS"):   # threadpool_limits(1)
        os.environ[var] = "1"
    _PGRAM, _KIND, what = _load_pgram()
    if _A.workload == "cfg5":
        with open(_A.files_from) as f:
            _FILES = [l.strip() for l in f if l.strip()]
        ntrials = min(len(_FILES), cores * _A.trials_per_core)
        work, unit = _file, "SIGPROC file(s) of cfg5 (2^23 samples @ 64 us), read + 3 example.yaml ranges"
    else:
        ntrials = cores * _A.trials_per_core
        work = _trial
        c = WORKLOADS[_A.workload]
        unit = f"{_A.workload} trial(s) of {c['n']} samples"
    ctx = multiprocessing.get_context("fork")
    with ctx.Pool(processes=cores) as pool:
        stamps = pool.map(work, range(ntrials), chunksize=1)
    start = min(s[0] for s in stamps)
    search_wall = max(s[1] for s in stamps) - start
    total_wall = max(s[2] for s in stamps) - start
    print(json.dumps({
        "value": ntrials / search_wall, "unit": "DM trials/s", "cores": cores, "kind": _KIND,
        "search_and_peaks_per_s": ntrials / total_wall,
        "per_core_search_per_s": ntrials / search_wall / cores,
        "sample": f"{ntrials} {unit}, multiprocessing.Pool({cores}) one trial per process (rffa worker-pool "
                  f"model): numpy deredden+normalise + {what} periodogram = value; + find_peaks = "
                  f"search_and_peaks_per_s; {affinity} affinity cores on this host"
                  + (f", cgroup CPU quota {quota:g} cores" if quota else "")
                  + (f", workers capped at {mem_cap} by available memory" if mem_cap and mem_cap < affinity else ""),
        "affinity_cores": affinity, "cpu_quota_cores": quota,
        "seconds": total_wall}))


if __name__ == "__main__":
    main()
